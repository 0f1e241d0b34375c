"""CPU: the C-ABI library loads and exports exactly what include/kdpc.h declares, and
rejects invalid sizes with hipErrorInvalidValue before touching a device."""
import ctypes
import os
import re

import pytest

import kdpc_native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "kdpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kdpc_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = kdpc_native.load_library()
    declared = _declared()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(kdpc_native.EXPORTED) == declared


def test_exported_symbols_are_only_the_abi():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", kdpc_native.LIB_PATH],
                         capture_output=True, text=True).stdout
    ours = sorted(set(re.findall(r"\b(kdpc_\w+)$", out, flags=re.M)))
    assert ours == _declared()


def test_invalid_sizes_rejected_without_launch():
    lib = kdpc_native.load_library()
    EINVAL = 1  # hipErrorInvalidValue
    assert lib.kdpc_knn_point(1, 10, 5, 0, None, None, None, None, None) == EINVAL  # k=0
    assert lib.kdpc_knn_point(1, 10, 5, 65, None, None, None, None, None) == EINVAL  # k>64
    assert lib.kdpc_knn_point(1, 10, 5, 11, None, None, None, None, None) == EINVAL  # k>n
    assert lib.kdpc_furthest_point_sampling(1, 0, 5, None, None, None, None) == EINVAL
    assert lib.kdpc_group_points(-1, 1, 1, 1, 1, None, None, None, None) == EINVAL
    assert lib.kdpc_csr_workspace_bytes(0, 10, 10) == 0
    # empty work is a successful no-op
    assert lib.kdpc_gather_points(0, 3, 10, 4, None, None, None, None) == 0


def test_opt_n_threads_matches_reference_rule():
    lib = kdpc_native.load_library()
    import pointnet2_oracle as O
    for n in (1, 2, 3, 63, 64, 100, 512, 1000, 1024, 4096, 8192, 100000):
        assert lib.kdpc_opt_n_threads(n) == O.opt_n_threads(n)


def _declared_arity():
    src = open(os.path.join(ROOT, "include", "kdpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(kdpc_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        params = [p for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        out[m.group(1)] = params
    return out


def test_ctypes_signatures_match_header():
    """Every ctypes binding passes exactly the header's parameters, with matching kinds
    (pointer / size_t / float / double / long long / int)."""
    decl = _declared_arity()
    for name, argtypes in kdpc_native._SIGNATURES.items():
        params = decl[name]
        assert len(params) == len(argtypes), (name, len(params), len(argtypes))
        for p, t in zip(params, argtypes):
            p = p.strip()
            if "*" in p:
                assert t is ctypes.c_void_p, (name, p)
            elif p.startswith("size_t"):
                assert t is ctypes.c_size_t, (name, p)
            elif p.startswith("float"):
                assert t is ctypes.c_float, (name, p)
            elif p.startswith("double"):
                assert t is ctypes.c_double, (name, p)
            elif p.startswith("long long"):
                assert t is ctypes.c_longlong, (name, p)
            else:
                assert t is ctypes.c_int, (name, p)


def test_library_built_from_these_sources():
    """kdpc_build_id() is the hash of the sources next to the library, of the arch + flags and
    of the hipcc version: the loader refuses a stale binary (a changed kernel source without
    a rebuild) and one built for another arch or with other flags."""
    import build_native
    lib = kdpc_native.load_library()
    assert lib.kdpc_build_id().decode() == build_native.build_id()
    assert build_native._lib_current(build_native.build_id())


def test_other_arch_or_flags_change_the_build_id(monkeypatch):
    """Rebuilding for another arch (KDPC_ARCH) or with other flags must not reuse the shipped
    library (the id used to cover the sources only)."""
    import build_native
    base = build_native.build_id(tool="hipcc x")
    monkeypatch.setattr(build_native, "ARCH", "gfx942")
    assert build_native.build_id(tool="hipcc x") != base
    assert not build_native._lib_current(build_native.build_id())
    monkeypatch.undo()
    monkeypatch.setattr(build_native, "EXTRA_FLAGS", {"fps.hip": ["-O1"]})
    assert build_native.build_id(tool="hipcc x") != base
    monkeypatch.undo()
    assert build_native.build_id(tool="hipcc y") != base
    assert build_native.build_id(tool="hipcc x") == base


def test_stale_library_is_refused(tmp_path):
    import build_native
    import shutil
    csrc = tmp_path / "csrc"
    shutil.copytree(build_native.CSRC, csrc)
    (tmp_path / "include").mkdir()
    shutil.copy(os.path.join(ROOT, "include", "kdpc.h"), tmp_path / "include")
    assert build_native.source_id(str(csrc), str(tmp_path)) == build_native.source_id()
    with open(csrc / "fps.hip", "a") as f:
        f.write("\n// edited\n")
    assert build_native.source_id(str(csrc), str(tmp_path)) != build_native.source_id()


# every torch operator torch_ops/kdpc_torch_ops.cpp registers -> the C entry point it calls
TORCH_OPS = {
    "ball_query_wrapper": "kdpc_ball_query", "group_points_wrapper": "kdpc_group_points",
    "group_points_grad_wrapper": "kdpc_group_points_grad_ws",
    "gather_points_wrapper": "kdpc_gather_points",
    "gather_points_grad_wrapper": "kdpc_gather_points_grad_ws",
    "furthest_point_sampling_wrapper": "kdpc_furthest_point_sampling",
    "three_nn_wrapper": "kdpc_three_nn", "three_interpolate_wrapper": "kdpc_three_interpolate",
    "three_interpolate_grad_wrapper": "kdpc_three_interpolate_grad_ws",
    "furthest_point_sample": "kdpc_furthest_point_sampling", "gather_points": "kdpc_gather_points",
    "ball_query": "kdpc_ball_query", "group_points": "kdpc_group_points",
    "three_nn": "kdpc_three_nn", "three_interpolate": "kdpc_three_interpolate",
    "knn_point": "kdpc_knn_point_ws", "knn_point_dist": "kdpc_knn_point_ws",
    "knn_feature": "kdpc_knn_feature", "knn_feature_dist": "kdpc_knn_feature",
    "group_rows": "kdpc_group_rows", "csr_build": "kdpc_csr_build",
    "group_rows_grad": "kdpc_group_rows_grad_csr", "csr_sum_channels": "kdpc_csr_sum_channels",
    "three_interpolate_grad_csr": "kdpc_three_interpolate_grad_csr",
    "cost_volume_fwd": "kdpc_cost_volume_fwd", "cost_volume_bwd": "kdpc_cost_volume_bwd",
    "cost_volume_bwd_csr": "kdpc_cost_volume_bwd_csr", "csr_rank": "kdpc_csr_rank",
    "cost_volume_wide_h0": "kdpc_cost_volume_wide_h0",
    "cost_volume_wide_max": "kdpc_cost_volume_wide_max",
    "cost_volume_wide_max_bwd": "kdpc_cost_volume_wide_max_bwd",
    "cost_volume_wide_h0_bwd": "kdpc_cost_volume_wide_h0_bwd",
    "pointconv_fwd": "kdpc_pointconv_fwd", "pointconv_bwd": "kdpc_pointconv_bwd",
    "pointconv_bwd_data": "kdpc_pointconv_bwd_data",
    "pointconv_bwd_weight": "kdpc_pointconv_bwd_weight",
    "pointconv_contract_fwd": "kdpc_pointconv_contract_fwd",
    "pointconv_contract_bwd": "kdpc_pointconv_contract_bwd",
    "weightnet_fwd": "kdpc_weightnet_fwd", "weightnet_bwd": "kdpc_weightnet_bwd",
    "weightnet_bwd_rel": "kdpc_weightnet_bwd_rel",
    "wn_wsum_fwd": "kdpc_wn_wsum_fwd", "wn_wsum_bwd": "kdpc_wn_wsum_bwd",
    "batchnorm_lrelu_fwd": "kdpc_batchnorm_lrelu_fwd",
    "batchnorm_lrelu_apply": "kdpc_batchnorm_lrelu_apply",
    "batchnorm_lrelu_bwd": "kdpc_batchnorm_lrelu_bwd", "colsum": "kdpc_colsum",
    "idw_blend_fwd": "kdpc_idw_blend_fwd", "idw_blend_bwd_vals": "kdpc_idw_blend_bwd_vals",
    "idw_blend_bwd_coords": "kdpc_idw_blend_bwd_coords",
    "dense_tn_small": "kdpc_dense_tn_small", "dense_small": "kdpc_dense_small",
    "neg_sum_k": "kdpc_neg_sum_k",
    "copy_segments": "kdpc_copy_segments",
    "adam_step": "kdpc_adam_step",
    "morton_order": "kdpc_morton_order", "pc_tile_plan": "kdpc_pc_tile_plan",
    "pointconv_bwd_tiled": "kdpc_pointconv_bwd_tiled",
    "pointconv_fwd_tiled": "kdpc_pointconv_fwd_tiled",
    "pointconv_bwd_weight_bias": "kdpc_pointconv_bwd_weight_bias",
    "dense_small_out": "kdpc_dense_small",
}


def test_torch_op_library_registers_every_op():
    """torch.ops.kdpc loads (in a child process: a schema mismatch aborts at load time),
    registers every operator above with a GPU kernel and calls only declared C entry points
    (each one's definition is in the source)."""
    import subprocess
    import sys
    code = ("import sys, torch; sys.path.insert(0, %r); import kdpc_native as k; k.load_ops(); "
            "import torch._C as C; "
            "names = sorted(s.name[len('kdpc::'):] for s in C._jit_get_all_schemas() "
            "if s.name.startswith('kdpc::')); print(' '.join(names))"
            % os.path.join(ROOT, "kd-pointcloud_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(r.stdout.split()) == sorted(TORCH_OPS)
    src = open(os.path.join(ROOT, "kd-pointcloud_amd", "torch_ops", "kdpc_torch_ops.cpp")).read()
    declared = set(_declared())
    for op, entry in TORCH_OPS.items():
        assert entry in declared, (op, entry)
        assert entry + "(" in src, (op, entry)


def test_torch_ops_reject_cpu_tensors():
    import torch
    with pytest.raises(kdpc_native.KdpcError):
        kdpc_native.knn_point(4, torch.zeros(1, 16, 3), torch.zeros(1, 8, 3))
    ops = kdpc_native.load_ops()
    with pytest.raises(NotImplementedError):  # no CPU kernel is registered
        ops.group_rows(torch.zeros(1, 4, 3), torch.zeros(1, 2, dtype=torch.int32))


def test_library_holds_no_packed_f32_instructions(tmp_path):
    """No v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 / v_pk_mov_b32 in any gfx950 code object
    of the built library (kdpc_common.h: packed f32 results were wrong now and then beside
    another kernel's waves on the MI355X).  Disassembles a copy of the
    library (llvm-objdump --offloading writes the code objects next to its input)."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not installed")
    lib = tmp_path / "libkdpc_hip.so"
    shutil.copy(kdpc_native.LIB_PATH, lib)
    subprocess.run([objdump, "--offloading", str(lib)], check=True, capture_output=True)
    objs = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in the library"
    bad = {}
    for p in objs:
        text = subprocess.run([objdump, "-d", str(p)], check=True, capture_output=True,
                              text=True).stdout
        fn = None
        for line in text.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                fn = m.group(1)
            elif re.search(r"\bv_pk_(fma|mul|add)_f32\b|\bv_pk_mov_b32\b", line):
                bad[fn] = bad.get(fn, 0) + 1
    assert not bad, f"packed f32 instructions in: {sorted(bad.items())[:8]}"
