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
    (pointer / size_t / float / int)."""
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
            else:
                assert t is ctypes.c_int, (name, p)


def test_library_built_from_these_sources():
    """kdpc_build_id() is the hash of the sources next to the library: the loader refuses a
    stale binary (a changed kernel source without a rebuild)."""
    import build_native
    lib = kdpc_native.load_library()
    assert lib.kdpc_build_id().decode() == build_native.source_id()


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
