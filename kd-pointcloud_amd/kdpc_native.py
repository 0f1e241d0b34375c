"""Python face of the gfx950 HIP kernels for torch-ROCm tensors.

Two layers over libkdpc_hip.so (the C ABI in include/kdpc.h):
  * torch.ops.kdpc (lib/libkdpc_torch.so, torch_ops/kdpc_torch_ops.cpp): every C entry
    point registered as a torch operator with a schema, TORCH_CHECKed inputs, outputs and
    scratch from the caching allocator, launched on the current torch stream.  Every op
    function below goes through it;
  * a ctypes binding of the bare C ABI (load_library, _SIGNATURES), used by the C-ABI
    tests (export / arity / argument validation) and by build-id verification.
There is no CPU path: a missing library or a CPU tensor raises.
"""
import ctypes
import functools
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KDPC_LIB", os.path.join(_HERE, "lib", "libkdpc_hip.so"))
OPS_PATH = os.path.join(os.path.dirname(LIB_PATH), "libkdpc_torch.so")

_c_int, _c_float, _c_size, _vp = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
_c_double, _c_longlong = ctypes.c_double, ctypes.c_longlong

# name -> argtypes (all return int hipError_t, except where noted)
_SIGNATURES = {
    "kdpc_furthest_point_sampling": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_opt_n_threads": [_c_int],
    "kdpc_gather_points": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_gather_points_grad": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_grad_workspace_bytes": [_c_int, _c_int, _c_int],
    "kdpc_gather_points_grad_ws": [_c_int] * 4 + [_vp] * 4 + [_c_size, _vp],
    "kdpc_group_points_grad_ws": [_c_int] * 5 + [_vp] * 4 + [_c_size, _vp],
    "kdpc_three_interpolate_grad_ws": [_c_int] * 4 + [_vp] * 5 + [_c_size, _vp],
    "kdpc_build_id": [],
    "kdpc_ball_query": [_c_int, _c_int, _c_int, _c_float, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_group_points": [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_group_points_grad": [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_three_nn": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_three_interpolate": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_three_interpolate_grad": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_knn_point": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_knn_workspace_bytes": [_c_int] * 3,
    "kdpc_cost_volume_wide_supported": [_c_int] * 3,
    "kdpc_cost_volume_wide_h0": [_c_int] * 5 + [_vp] * 9,
    "kdpc_cost_volume_wide_max": [_c_int] * 4 + [_vp] * 4,
    "kdpc_cost_volume_wide_max_bwd": [_c_int] * 4 + [_vp] * 6,
    "kdpc_cost_volume_wide_slab_rows": [],
    "kdpc_cost_volume_wide_h0_bwd": [_c_int] * 5 + [_vp] * 8,
    "kdpc_knn_point_ws": [_c_int] * 4 + [_vp] * 5 + [_c_size, _vp],
    "kdpc_knn_point_evals": [_c_int] * 4 + [_vp] * 4 + [_c_size, _vp, _vp],
    "kdpc_group_rows": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_csr_workspace_bytes": [_c_int, _c_int, _c_int],
    "kdpc_csr_build": [_c_int, _c_int, _c_int, _vp, _vp, _c_size, _vp, _vp, _vp],
    "kdpc_group_rows_grad_csr": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_csr_rank": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_csr_sum_channels": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_three_interpolate_grad_csr": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp,
                                        _vp, _vp],
    "kdpc_cost_volume_fwd": [_c_int] * 6 + [_vp] * 12,
    "kdpc_pointconv_contract_fwd": [_c_int] * 5 + [_vp] * 7,
    "kdpc_pointconv_contract_bwd": [_c_int] * 5 + [_vp] * 10,
    "kdpc_cost_volume_bwd_workspace_bytes": [_c_int] * 4,
    "kdpc_cost_volume_bwd": [_c_int] * 6 + [_vp] * 17 + [_c_size, _vp, _vp],
    "kdpc_cost_volume_bwd_csr_workspace_bytes": [_c_int] * 5,
    "kdpc_cost_volume_bwd_csr": [_c_int] * 6 + [_vp] * 19 + [_c_size, _vp, _vp],
    "kdpc_pointconv_supported": [_c_int] * 3,
    "kdpc_pointconv_fwd_workspace_bytes": [_c_int] * 5,
    "kdpc_pointconv_fwd": [_c_int] * 6 + [_vp] * 9 + [_c_size, _vp],
    "kdpc_pointconv_fwd_tiled": [_c_int] * 6 + [_vp] * 8 + [_c_int, _vp, _vp, _c_size, _vp],
    "kdpc_pointconv_bwd_workspace_bytes": [_c_int] * 5,
    "kdpc_pointconv_bwd": [_c_int] * 6 + [_vp] * 15 + [_c_size, _vp],
    "kdpc_pointconv_bwd_data": [_c_int] * 6 + [_vp] * 14 + [_c_size, _vp],
    "kdpc_pointconv_bwd_data_tiled": [_c_int] * 6 + [_vp] * 17 + [_c_size, _vp],
    "kdpc_pointconv_bwd_tiled": [_c_int] * 6 + [_vp] * 18 + [_c_size, _vp],
    "kdpc_morton_order": [_c_int, _c_int, _vp, _vp, _vp],
    "kdpc_pointconv_bwd_weight_bias": [_c_int] * 6 + [_vp] * 9 + [_c_size, _vp],
    "kdpc_pc_tile_plan": [_c_int] * 4 + [_vp] * 7,
    "kdpc_pointconv_bwd_weight_workspace_bytes": [_c_int] * 5,
    "kdpc_pointconv_bwd_weight": [_c_int] * 6 + [_vp] * 8 + [_c_size, _vp],
    "kdpc_batchnorm_workspace_bytes": [_c_int, _c_int],
    "kdpc_batchnorm_lrelu_fwd": [_c_int, _c_int] + [_vp] * 3 + [_c_float] * 3 + [_vp] * 6
                                + [_c_size, _vp],
    "kdpc_batchnorm_lrelu_apply": [_c_int, _c_int] + [_vp] * 5 + [_c_float, _vp, _vp],
    "kdpc_batchnorm_lrelu_bwd": [_c_int, _c_int] + [_vp] * 6 + [_c_float] + [_vp] * 4
                                + [_c_size, _vp],
    "kdpc_colsum_workspace_bytes": [_c_int, _c_int],
    "kdpc_colsum": [_c_int, _c_int, _vp, _vp, _vp, _c_size, _vp],
    "kdpc_neg_sum_k": [_c_int, _c_int, _c_int, _vp, _vp, _vp],
    "kdpc_copy_segments": [_c_int, _vp, _vp, _vp, _vp],
    "kdpc_adam_step": [_c_longlong, _vp, _vp, _vp, _vp, _vp, _vp, _c_double, _c_double,
                       _c_double, _c_double, _c_int, _c_int, _vp],
    "kdpc_weightnet_param_count": [],
    "kdpc_weightnet_fwd": [_c_int] * 4 + [_vp] * 11,
    "kdpc_weightnet_bwd_workspace_bytes": [],
    "kdpc_weightnet_bwd": [_c_int] * 4 + [_vp] * 13 + [_c_size, _vp],
    "kdpc_weightnet_bwd_rel": [_c_int] * 4 + [_vp] * 12,
    "kdpc_knn_feature_workspace_bytes": [_c_int] * 3,
    "kdpc_knn_feature": [_c_int] * 5 + [_vp] * 5 + [_c_size, _vp],
    "kdpc_wn_wsum_param_count": [_c_int],
    "kdpc_wn_wsum_fwd": [_c_int] * 5 + [_vp] * 11,
    "kdpc_wn_wsum_bwd_workspace_bytes": [_c_int] * 3,
    "kdpc_wn_wsum_bwd": [_c_int] * 5 + [_vp] * 14 + [_c_size, _vp],
    "kdpc_idw_blend_fwd": [_c_int] * 4 + [_vp] * 6 + [_c_int, _vp],
    "kdpc_idw_blend_bwd_vals": [_c_int] * 4 + [_vp] * 5 + [_c_int, _vp],
    "kdpc_idw_blend_bwd_coords": [_c_int] * 4 + [_vp] * 7 + [_c_int, _vp],
    "kdpc_dense_tn_small_workspace_bytes": [_c_int] * 3,
    "kdpc_dense_tn_small": [_c_int] * 3 + [_vp] * 4 + [_c_size, _vp],
    "kdpc_dense_small": [_c_int] * 3 + [_vp] * 5,
}
_RESTYPES = {"kdpc_build_id": ctypes.c_char_p, "kdpc_grad_workspace_bytes": _c_size,
             "kdpc_csr_workspace_bytes": _c_size, "kdpc_cost_volume_bwd_workspace_bytes": _c_size,
             "kdpc_cost_volume_bwd_csr_workspace_bytes": _c_size,
             "kdpc_pointconv_fwd_workspace_bytes": _c_size,
             "kdpc_pointconv_bwd_workspace_bytes": _c_size,
             "kdpc_pointconv_bwd_weight_workspace_bytes": _c_size,
             "kdpc_weightnet_bwd_workspace_bytes": _c_size,
             "kdpc_wn_wsum_bwd_workspace_bytes": _c_size,
             "kdpc_knn_feature_workspace_bytes": _c_size,
             "kdpc_batchnorm_workspace_bytes": _c_size,
             "kdpc_colsum_workspace_bytes": _c_size, "kdpc_knn_workspace_bytes": _c_size,
             "kdpc_dense_tn_small_workspace_bytes": _c_size}

EXPORTED = tuple(_SIGNATURES)

_lib = None


class KdpcError(RuntimeError):
    pass


def load_library(path=LIB_PATH):
    """Load and type the HIP library (works without a GPU: symbols only)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KdpcError(
            f"kd-pointcloud_amd HIP library not found at {path}; build it with "
            "`python kd-pointcloud_amd/build_native.py` (there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, args in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, _c_int)
    _check_build_id(lib, path)
    _lib = lib
    return lib


def _check_build_id(lib, path):
    """The library must have been built from the sources next to it (build_native.py embeds
    their hash): a stale binary is refused, so no run uses kernels its tree does not hold.
    Skipped when the sources are not shipped (KDPC_LIB pointing at an installed library)."""
    if not os.path.isdir(os.path.join(_HERE, "csrc")) or os.environ.get("KDPC_LIB"):
        return
    import build_native
    want = build_native.source_id()
    got = lib.kdpc_build_id().decode().split("+")
    if got[0] != want:
        raise KdpcError(f"{path} was built from other sources (build id {got[0][:12]}, sources "
                        f"{want[:12]}); rebuild with `python kd-pointcloud_amd/build_native.py`")
    if len(got) < 2 or got[1] != build_native.flags_id():
        raise KdpcError(f"{path} was built for another arch or with other flags (KDPC_ARCH="
                        f"{build_native.ARCH}); rebuild with `python kd-pointcloud_amd/"
                        "build_native.py`")


def _check(status, name):
    if status != 0:
        raise KdpcError(f"{name} failed with hipError_t {status}")


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _dev(t, dtype, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if not t.is_cuda:
        raise KdpcError(f"{name} must be a GPU (HIP) tensor: kd-pointcloud_amd has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t.data_ptr()


class LaunchTimer:
    """Brackets every launch of the named C entry points with HIP events on the current
    torch stream (the stream the kernel runs on) and accumulates per-launch algorithmic
    bytes/flops supplied by the op wrappers.  Used by bench.py for the live roofline."""

    def __init__(self, names, lead_cycles=0):
        self.names = set(names)
        self.records = []  # (name, start_event, end_event, bytes, flops)
        # a GPU spin of this many cycles before each bracketed launch: the host then enqueues
        # the start event, the entry's kernels and the end event while the GPU is busy, so a
        # host-bound step's issue gaps do not land inside the bracket
        self.lead_cycles = lead_cycles

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, nbytes, flops in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0.0, "flops": 0.0})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["bytes"] += nbytes
            d["flops"] += flops
        return out


_timer = None


def set_launch_timer(timer):
    global _timer
    _timer = timer


def _call(name, *args, work=None):
    """Invoke a C entry point through ctypes (C-ABI tests); `work` as for _op."""
    lib = load_library()
    t = _timer
    if t is not None and name in t.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        _check(getattr(lib, name)(*args), name)
        e1.record()
        nb, fl = work if work is not None else (0.0, 0.0)
        t.records.append((name, e0, e1, float(nb), float(fl)))
        return
    _check(getattr(lib, name)(*args), name)


_ops = None


def load_ops():
    """torch.ops.kdpc, loaded once (after the C library's build-id check)."""
    global _ops
    if _ops is None:
        load_library()
        if not os.path.exists(OPS_PATH):
            raise KdpcError(f"kd-pointcloud_amd torch op library not found at {OPS_PATH}; build "
                            "it with `python kd-pointcloud_amd/build_native.py`")
        torch.ops.load_library(OPS_PATH)
        _ops = torch.ops.kdpc
    return _ops


def _gpu(t, name):
    if not t.is_cuda:
        raise KdpcError(f"{name} must be a GPU (HIP) tensor: kd-pointcloud_amd has no CPU path")
    return t


def _op(entry, op, *args, work=None):
    """Run torch.ops.kdpc.<op>; `entry` is the C entry point it launches (the unit the
    bench's live roofline brackets), `work` = (algorithmic bytes, flops) of the launch."""
    fn = getattr(_ops or load_ops(), op)
    t = _timer
    if t is not None and entry in t.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        if t.lead_cycles:
            torch.cuda._sleep(t.lead_cycles)
        e0.record()
        out = fn(*args)
        e1.record()
        nb, fl = work if work is not None else (0.0, 0.0)
        t.records.append((entry, e0, e1, float(nb), float(fl)))
        return out
    return fn(*args)


# ------------------------------------------------------------------------------ ops
def furthest_point_sampling(xyz, npoint, temp=None):
    """xyz (B,N,3) f32 -> idx (B,npoint) i32.  temp: optional (B,N) scratch (1e10-filled),
    left holding the final min-distances (the reference wrapper's in-place contract)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    work = (B * (12 * N + 8 * N + 4 * npoint), B * N * npoint * 8)
    if temp is None:
        return _op("kdpc_furthest_point_sampling", "furthest_point_sample", xyz, npoint,
                   work=work)
    idx = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
    _op("kdpc_furthest_point_sampling", "furthest_point_sampling_wrapper", B, N, npoint, xyz,
        temp, idx, work=work)
    return idx


def gather_points(points, idx):
    """points (B,C,N), idx (B,M) i32 -> (B,C,M)."""
    return _op("kdpc_gather_points", "gather_points", _gpu(points, "points"), idx)


def ball_query(radius, nsample, xyz, new_xyz):
    return _op("kdpc_ball_query", "ball_query", float(radius), int(nsample), _gpu(xyz, "xyz"),
               new_xyz)


def group_points(points, idx):
    """points (B,C,N), idx (B,S,K) i32 -> (B,C,S,K)."""
    B, C, N = _gpu(points, "points").shape
    _, S, K = idx.shape
    # SURVEY §8d algorithmic bytes: B*(4CN + 4SK + 4CSK)
    return _op("kdpc_group_points", "group_points", points, idx,
               work=(B * (4 * C * N + 4 * S * K + 4 * C * S * K), 0))


def three_nn(unknown, known):
    """-> (dist2 (B,N,3) squared, idx (B,N,3) i32)."""
    return _op("kdpc_three_nn", "three_nn", _gpu(unknown, "unknown"), known)


def three_interpolate(points, idx, weight):
    return _op("kdpc_three_interpolate", "three_interpolate", _gpu(points, "points"), idx,
               weight)


def knn_point(nsample, xyz, new_xyz, return_dist=False, seeded=True):
    """xyz (B,N,3) refs, new_xyz (B,S,3) queries -> idx (B,S,K) i32 ascending (dist, idx).
    seeded: allow the seeded-threshold scan where it pays (identical results; False forces
    the unseeded scan, for tests)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S = new_xyz.shape[1]
    if nsample > N:
        raise ValueError(f"knn_point: nsample={nsample} > number of points {N}")
    work = (B * (12 * N + 12 * S + 4 * S * nsample * (2 if return_dist else 1)), B * S * N * 8)
    if return_dist:
        return _op("kdpc_knn_point", "knn_point_dist", int(nsample), xyz, new_xyz, seeded,
                   work=work)
    return _op("kdpc_knn_point", "knn_point", int(nsample), xyz, new_xyz, seeded, work=work)


def knn_point_evals(nsample, xyz, new_xyz):
    """The culled kNN scan through the bare C ABI (kdpc_knn_point_evals) -> (idx (B,S,K) i32,
    number of query-ref distance evaluations it issued).  Measurement only (bench.py's
    configs[4] roofline): the same indices as knn_point; needs a problem large enough for the
    culled path."""
    lib = load_library()
    B, N, _ = _gpu(xyz, "xyz").shape
    S = new_xyz.shape[1]
    ws_bytes = lib.kdpc_knn_workspace_bytes(B, N, S)
    if ws_bytes == 0:
        raise KdpcError("knn_point_evals: the problem is too small for the culled scan")
    xyz, new_xyz = xyz.contiguous(), new_xyz.contiguous()
    idx = torch.empty((B, S, nsample), dtype=torch.int32, device=xyz.device)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=xyz.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=xyz.device)
    _check(lib.kdpc_knn_point_evals(B, N, S, int(nsample), xyz.data_ptr(), new_xyz.data_ptr(),
                                    idx.data_ptr(), ws.data_ptr(), ws_bytes, cnt.data_ptr(),
                                    _stream(xyz)), "kdpc_knn_point_evals")
    return idx, int(cnt.item())


def knn_feature(nsample, ref, query, return_dist=False):
    """kNN in feature space: ref (B,N,D), query (B,S,D), D <= 128 -> idx (B,S,K) i32
    ascending (dist, idx) [, dist]; the distance GEMM runs on the f32 matrix cores."""
    B, N, D = _gpu(ref, "ref").shape
    S = query.shape[1]
    if nsample > N:
        raise ValueError(f"knn_feature: nsample={nsample} > number of points {N}")
    work = (B * 4 * (N * D + S * D + S * nsample * (2 if return_dist else 1)),
            2.0 * B * S * N * D)
    if return_dist:
        return _op("kdpc_knn_feature", "knn_feature_dist", int(nsample), ref.contiguous(),
                   query.contiguous(), work=work)
    return _op("kdpc_knn_feature", "knn_feature", int(nsample), ref.contiguous(),
               query.contiguous(), work=work)


def group_rows(points, idx):
    """points (B,N,C), idx (B,P) i32 -> (B,P,C) (point-major row gather)."""
    B, N, C = _gpu(points, "points").shape
    P = idx.shape[1]
    # algorithmic bytes: table read once + idx read + rows written
    return _op("kdpc_group_rows", "group_rows", points, idx,
               work=(B * (4 * N * C + 4 * P + 4 * P * C), 0))


class Csr:
    """Inverted index of an int32 index tensor (B,P) over a key space of n values."""
    __slots__ = ("offsets", "perm", "n", "p", "rank")

    def __init__(self, idx2d, n):
        self.offsets, self.perm = _op("kdpc_csr_build", "csr_build", _gpu(idx2d, "idx"), n)
        self.n, self.p = n, idx2d.shape[1]
        self.rank = None


def batch_prefix(idx, b):
    """idx[:b] (the first b batch entries) whose CSR is derived from idx's own: keys are
    batch-major (b*N + idx), so the inverted index of the first b batches is exactly the
    prefix offsets[:b*N+1], perm[:b*P] of the parent's -- no second sort."""
    child = idx[:b]
    try:
        child._kdpc_parent = (idx, b)
    except AttributeError:
        pass
    return child


def csr_of(idx, n):
    """CSR for idx (B,...) flattened to (B,P), cached on the index tensor object."""
    cache = getattr(idx, "_kdpc_csr", None)
    if cache is not None and cache.n == n:
        return cache
    parent = getattr(idx, "_kdpc_parent", None)
    if parent is not None:
        pidx, b = parent
        pc = csr_of(pidx, n)
        csr = Csr.__new__(Csr)
        csr.offsets, csr.perm = pc.offsets[:b * n + 1], pc.perm[:b * pc.p]
        csr.n, csr.p = n, pc.p
        csr.rank = None
    else:
        csr = Csr(idx.reshape(idx.shape[0], -1), n)
    try:
        idx._kdpc_csr = csr
    except AttributeError:
        pass
    return csr


def attach_csr(idx, n, offsets, perm, rank=None):
    """Cache an inverted index built elsewhere (e.g. on a prefetch stream:
    PointConvBidirection.precompute_plan) on the index tensor object, as csr_of /
    csr_rank_of would have: offsets (B*n+1), perm (B*P)[, rank (B*P)] of idx (B, ...)."""
    p = idx[0].numel() if idx.shape[0] else 0
    if offsets.numel() != idx.shape[0] * n + 1 or perm.numel() != idx.numel() or \
            (rank is not None and rank.numel() != idx.numel()):
        raise ValueError("attach_csr: CSR sizes do not match the index tensor")
    csr = Csr.__new__(Csr)
    csr.offsets, csr.perm, csr.rank = offsets, perm, rank
    csr.n, csr.p = n, p
    idx._kdpc_csr = csr
    return csr


def csr_rank_of(idx, n):
    """The CSR of idx (csr_of) with its inverse permutation: rank (B*P) int32, the slot of
    every position (perm[rank[i]] == i), built once and cached with the CSR.  A batch prefix
    (batch_prefix) takes the parent's prefix: slots of the first b batches are < offsets[b*N]."""
    csr = csr_of(idx, n)
    if csr.rank is None:
        parent = getattr(idx, "_kdpc_parent", None)
        if parent is not None:
            pidx, b = parent
            csr.rank = csr_rank_of(pidx, n).rank[:b * csr.p]
        else:
            idx2d = idx.reshape(idx.shape[0], -1)
            csr.rank = _op("kdpc_csr_rank", "csr_rank", _gpu(idx2d, "idx"), csr.offsets,
                           csr.perm, n)
    return csr


# ------------------------------------------------------------- tiled PointConv backward
# The PointConv backward with the dG rows summed per (32-row tile, destination) inside the
# data kernel (csrc/tile_plan.hip, pointconv_fused.hip): rows of a tile in Morton order of
# their centers, so their 32K neighbours name few distinct points (self-kNN K=9: ~69 of 288
# at N=8192).  Used for K <= 9 (the estimators' layers).  The three switches below are test
# seams (the tests compare each path with its untiled / unfused counterpart), not settings.
TILED_PC = True
# the PointConv bias gradient from the weight kernel's MFMAs (False: the fixed-order column
# sum of dy)
BIAS_IN_WEIGHT = True
# the forward through the same row tiles (bit-identical)
TILED_FWD = True
# K = 16 (the encoder layers) through the tiles measured slower: 13.60-13.80 -> 14.28-14.36 ms
# per train step (round 6, profiles/round06/rejected/tiled_max_k_*)
TILED_MAX_K = 9


class TilePlan:
    """Per-tile rows / sorted pairs / destination starts, plus the CSR of the partial rows
    (offsets over the B*n points, tdst = the partial-row slot of every (tile, destination))."""
    __slots__ = ("trow", "tpair", "tsoff", "offsets", "tdst", "n")


def tiled_supported(idx, center):
    return TILED_PC and idx.shape[-1] <= TILED_MAX_K and center.shape[1] <= 8192


def tile_plan_of(idx, center, n):
    """The tile plan of idx (B,S,K) over n points with rows ordered by their centers (B,S,3),
    cached on the index tensor object (a batch prefix takes its parent's tiles)."""
    tp = getattr(idx, "_kdpc_tplan", None)
    if tp is not None and tp.n == n:
        return tp
    parent = getattr(idx, "_kdpc_parent", None)
    if parent is not None:
        pidx, b = parent
        pp = getattr(pidx, "_kdpc_tplan", None)
        if pp is not None and pp.n == n:
            nt = b * ((idx.shape[1] + 31) // 32)
            tp = TilePlan()
            tp.trow, tp.tpair, tp.tsoff = pp.trow[:nt], pp.tpair[:nt], pp.tsoff[:nt]
            # tdst is (B, tiles per element * 32K): the prefix's partial-row slots
            tp.offsets, tp.tdst = pp.offsets[:b * n + 1], pp.tdst[:b]
            tp.n = n
            idx._kdpc_tplan = tp
            return tp
    idx = _gpu(idx, "idx")
    order = _op("kdpc_morton_order", "morton_order", _gpu(center, "center").contiguous())
    trow, tpair, tsoff, tkey = _op("kdpc_pc_tile_plan", "pc_tile_plan", idx, order, n)
    offsets, perm = _op("kdpc_csr_build", "csr_build", tkey, n)
    tdst = _op("kdpc_csr_rank", "csr_rank", tkey, offsets, perm, n)
    return attach_tile_plan(idx, n, trow, tpair, tsoff, offsets, tdst)


def tile_rows_of(idx, center, n):
    """The row order of the tiled forward only (trow: the Morton-ordered rows of every 32-row
    tile): a forward without gradients needs nothing else of the plan, so the CSR of the
    partial rows is not built for it.  A full plan cached on idx is used as it is."""
    if torch.is_grad_enabled():
        return tile_plan_of(idx, center, n).trow
    tp = getattr(idx, "_kdpc_tplan", None)
    if tp is not None and tp.n == n:
        return tp.trow
    order = _op("kdpc_morton_order", "morton_order", _gpu(center, "center").contiguous())
    return _op("kdpc_pc_tile_plan", "pc_tile_plan", _gpu(idx, "idx"), order, n)[0]


def attach_tile_plan(idx, n, trow, tpair, tsoff, offsets, tdst):
    """Cache a tile plan built elsewhere (PointConvBidirection.precompute_plan) on idx.
    tdst is kept as (B, tiles per element * 32K), the layout a batch prefix slices."""
    B, S, K = idx.shape
    nt = B * ((S + 31) // 32)
    if trow.shape != (nt, 32) or tpair.shape != (nt, 32 * K) or \
            tsoff.shape != (nt, 32 * K + 1) or offsets.numel() != B * n + 1 or \
            tdst.numel() != nt * 32 * K:
        raise ValueError("attach_tile_plan: plan sizes do not match the index tensor")
    tp = TilePlan()
    tp.trow, tp.tpair, tp.tsoff, tp.offsets, tp.n = trow, tpair, tsoff, offsets, n
    tp.tdst = tdst.reshape(B, -1)
    try:
        idx._kdpc_tplan = tp
    except AttributeError:
        pass
    return tp


def tile_plan_tensors(tp):
    return [tp.trow, tp.tpair, tp.tsoff, tp.offsets, tp.tdst]


def pointconv_fwd_tiled(xyz, center, feats, idx, wt, wl, bias, trow):
    """pointconv_fwd with the rows of each tile from a tile plan's trow (bit-identical)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    O, C = wl.shape[0], 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_fwd", "pointconv_fwd_tiled", xyz, center, feats, idx, wt, wl,
               bias, trow, work=(4 * R * (K + K * C + 16 * K + O) + 4 * O * 16 * C,
                                    2.0 * R * K * C * 16 + 2.0 * R * 16 * C * O))


def pointconv_bwd_tiled(xyz, center, feats, idx, wt, wl, dy, tp, need_xyz=True, weight=True):
    """pointconv_bwd / pointconv_bwd_data (weight=False) through a tile plan ->
    (dxyz|None, dfeats, dcenter, dwt, dwl|None)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    O, C = wl.shape[0], 3 + feats.shape[2]
    R = B * S
    # timed under the untiled entries' labels: the bench's live roofline brackets "the
    # PointConv backward" whichever C entry point runs it (kdpc_pointconv_bwd(_data)_tiled)
    entry = "kdpc_pointconv_bwd" if weight else "kdpc_pointconv_bwd_data"
    return _op(entry, "pointconv_bwd_tiled", xyz, center, feats, idx, wt, wl, dy,
               tp.offsets, tp.trow, tp.tpair, tp.tsoff, tp.tdst, bool(need_xyz), bool(weight),
               work=(4 * R * (2 * K * C + 32 * K + (2 if weight else 1) * O) +
                     (8 if weight else 4) * O * 16 * C,
                     4.0 * R * K * C * 16 + (4.0 if weight else 2.0) * R * 16 * C * O))


def group_rows_grad(grad_out, csr, B, N, C):
    """grad_out (B,P,C) -> (B,N,C) deterministic scatter-add through csr."""
    grad_out = grad_out.contiguous()
    P = grad_out.shape[1]
    return _op("kdpc_group_rows_grad_csr", "group_rows_grad", grad_out.view(B, P, C),
               csr.offsets, csr.perm, N, work=(B * (4 * P * C + 4 * P + 4 * N + 4 * N * C), 0))


def csr_sum_channels(src, csr, B, C, N):
    """src (B,C,P) -> (B,C,N): the backward of gather_points/group_points."""
    return _op("kdpc_csr_sum_channels", "csr_sum_channels", src.contiguous(), csr.offsets,
               csr.perm, B, C, N)


def three_interpolate_grad(grad_out, idx, weight, m):
    """grad_out (B,C,N) -> (B,C,M) deterministic."""
    csr = csr_of(idx, m)
    return _op("kdpc_three_interpolate_grad_csr", "three_interpolate_grad_csr",
               grad_out.contiguous(), weight, csr.offsets, csr.perm, m)


# ------------------------------------------------------------------ fused cost volume
# Every model width runs a one-kernel-each-way path: Din, Dout in {32, 64} (cost_volume.hip)
# and Din = Dout in {128, 256} (the fused MFMA kernels of cost_volume_wide.hip: gather +
# position transform + LeakyReLU + the Din x Dout MLP + max/argmax in one forward kernel, no
# h0 / z1 in HBM; round 4 whole-step A/B 16.96 / 17.12 -> 16.63 / 16.60 ms against the
# BLAS-GEMM formulation, which stays for the other widths: cost_volume_wide_*).


def cost_volume_supported(din, dout, k):
    """Shapes kdpc_cost_volume_fwd/_bwd take: Din, Dout in {32, 64} (cost_volume.hip), plus
    Din = Dout in {128, 256} (the fused wide kernels of cost_volume_wide.hip); K <= 32."""
    narrow = din in (32, 64) and dout in (32, 64)
    wide = din == dout and din in (128, 256)
    return (narrow or wide) and 1 <= k <= 32


def cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1):
    """-> out (B,N1,Dout) f32, amax (B,N1,Dout) u8.  See include/kdpc.h."""
    B, N1, _ = _gpu(x1, "x1").shape
    K = idx.shape[2]
    din, dout = p1.shape[2], w1.shape[0]
    # the wide shapes (the one-kernel MFMA path) are timed under their own label
    entry = "kdpc_cost_volume_fwd_wide" if din >= 128 else "kdpc_cost_volume_fwd"
    return _op(entry, "cost_volume_fwd", x1, x2, idx, p1, p2, wpos, bpos, w1,
               b1, work=(4 * B * N1 * (3 + K + din + K * din + 2 * dout) + B * N1 * dout,
                         2.0 * B * N1 * K * din * dout))


def cost_volume_bwd(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout, slope0=None):
    """-> dp1 (B,N1,Din), dp2_rows (B,N1,K,Din), dx1 (B,N1,3), ddir_rows (B,N1,K,3), dparams.
    slope0: optional (B,N1,K,Din) u8 override of the first LeakyReLU's derivative (test seam,
    include/kdpc.h)."""
    B, N1, _ = _gpu(x1, "x1").shape
    K = idx.shape[2]
    din, dout = p1.shape[2], w1.shape[0]
    # reads x1, idx, p1, the K gathered p2 rows, out, gout, amax; writes dp1, dp2_rows,
    # dx1, ddir_rows.  flops: dh0 = M W1 and dW1 = h0^T M over the K x Din x Dout tile
    return _op("kdpc_cost_volume_bwd", "cost_volume_bwd", x1, x2, idx, p1, p2,
               wpos, bpos, w1, out, amax, gout, slope0,
               work=(4 * B * N1 * (3 + K + din + K * din + 2 * dout + din + K * din + 3 + 3 * K)
                     + B * N1 * dout, 4.0 * B * N1 * K * din * dout))


def cost_volume_bwd_csr(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout, slope0=None):
    """-> dp1 (B,N1,Din), dp2 (B,N2,Din), dx1 (B,N1,3), dx2 (B,N2,3), dparams: the backward
    with the per-point sums through the (cached) CSR of idx done inside the entry point.
    slope0 as cost_volume_bwd."""
    B, N1, _ = _gpu(x1, "x1").shape
    N2, K = x2.shape[1], idx.shape[2]
    din, dout = p1.shape[2], w1.shape[0]
    csr = csr_rank_of(idx, N2)
    # reads x1, idx, rank, p1, the K gathered p2 rows, out, gout, amax, offsets; writes dp1,
    # dx1 and the per-point dp2 / dx2 (the CSR-ordered rows in between are not counted)
    entry = "kdpc_cost_volume_bwd_csr_wide" if din >= 128 else "kdpc_cost_volume_bwd_csr"
    return _op(entry, "cost_volume_bwd_csr", x1, x2, idx, p1, p2,
               wpos, bpos, w1, out, amax, gout, csr.offsets, csr.rank, slope0,
               work=(4 * B * N1 * (3 + 2 * K + din + K * din + 2 * dout + din + 3)
                     + B * N1 * dout + 4 * B * N2 * (din + 4) + 4,
                     4.0 * B * N1 * K * din * dout))


# ------------------------------------------------------------------ wide cost volume
@functools.lru_cache(maxsize=None)
def cost_volume_wide_supported(din, dout, k):
    return bool(load_library().kdpc_cost_volume_wide_supported(din, dout, k))


def cost_volume_wide_h0(x1, x2, idx, p1, p2, wpos, bpos):
    """-> h0 (B,N1,K,Din) = LeakyReLU(P2[idx] + P1 + Wpos dir + bpos)."""
    B, N1, _ = _gpu(x1, "x1").shape
    K, din = idx.shape[2], p1.shape[2]
    return _op("kdpc_cost_volume_wide_h0", "cost_volume_wide_h0", x1, x2, idx, p1, p2, wpos,
               bpos, work=(4 * B * N1 * (K * (1 + 2 * din + 3) + din + 3),
                           10.0 * B * N1 * K * din))


def cost_volume_wide_max(z1, B, N1, K, dout):
    """z1 (B*N1*K, Dout) -> out (B,N1,Dout), amax (B,N1,Dout) u8."""
    return _op("kdpc_cost_volume_wide_max", "cost_volume_wide_max", _gpu(z1, "z1"), B, N1, K,
               dout)


def cost_volume_wide_max_bwd(gout, out, amax, K):
    """-> dz1 (B*N1*K, Dout) dense, gsc (B*N1, Dout)."""
    return _op("kdpc_cost_volume_wide_max_bwd", "cost_volume_wide_max_bwd",
               _gpu(gout, "gout"), out, amax, K)


def cost_volume_wide_h0_bwd(x1, x2, idx, h0, dz, reduce=True):
    """dz (B*N1*K, Din) dh0 -> dz0 in place; -> dp1 (B,N1,Din), dWpos (Din,3) (reduce=False:
    the per-workgroup slab dWpos is the colsum(...).view(Din, 3) of)."""
    din = h0.shape[-1]
    dp1, slab = _op("kdpc_cost_volume_wide_h0_bwd", "cost_volume_wide_h0_bwd", _gpu(x1, "x1"),
                    x2, idx, h0, dz)
    return dp1, (colsum(slab).view(din, 3) if reduce else slab)


# ------------------------------------------------------------------ PointConv contraction
def pointconv_contract_fwd(xyz, center, feats, idx, wt):
    """-> A (B,S,16*(3+D)), c-major (the reference's .view(B,S,-1) of (B,S,C,16))."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    C = 3 + feats.shape[2]
    return _op("kdpc_pointconv_contract_fwd", "pointconv_contract_fwd", xyz, center, feats, idx,
               wt, work=(4 * B * S * (K + K * C + 16 * K + 16 * C), 2.0 * B * S * K * C * 16))


def pointconv_contract_bwd(xyz, center, feats, idx, wt, dout):
    """-> dg_rows (B,S,K,3+D), dwt (B,S,K,16), dcenter (B,S,3)."""
    return _op("kdpc_pointconv_contract_bwd", "pointconv_contract_bwd", _gpu(xyz, "xyz"),
               center, feats, idx, wt, dout)


# ------------------------------------------------------------------ fused PointConv layer
@functools.lru_cache(maxsize=None)
def pointconv_supported(k, d, o):
    return bool(load_library().kdpc_pointconv_supported(k, d, o))


def _workspace(nbytes, device):
    return torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device=device)


def pointconv_fwd(xyz, center, feats, idx, wt, wl, bias):
    """Fused gather + contraction + Linear: -> y (B,S,O) = A wl^T + bias, A never stored.
    xyz (B,N,3), center (B,S,3), feats (B,N,D), idx (B,S,K) i32, wt (B,S,K,16), wl (O,16C)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    O, C = wl.shape[0], 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_fwd", "pointconv_fwd", xyz, center, feats, idx, wt, wl, bias,
               work=(4 * R * (K + K * C + 16 * K + O) + 4 * O * 16 * C,
                     2.0 * R * K * C * 16 + 2.0 * R * 16 * C * O))


def pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=True):
    """Backward of pointconv_fwd for dy (B,S,O) -> (dxyz|None, dfeats, dcenter, dwt, dwl).
    csr: csr_rank_of(idx, N) (offsets + rank; a plain csr_of gets its rank built here)."""
    if csr.rank is None:
        csr = csr_rank_of(idx, xyz.shape[1])
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    O, C = wl.shape[0], 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_bwd", "pointconv_bwd", xyz, center, feats, idx, wt, wl, dy,
               csr.offsets, csr.rank, bool(need_xyz),
               work=(4 * R * (2 * K * C + 32 * K + 2 * O) + 8 * O * 16 * C,
                     4.0 * R * K * C * 16 + 4.0 * R * 16 * C * O))


def pointconv_bwd_data(xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=True):
    """Data half of pointconv_bwd -> (dxyz|None, dfeats, dcenter, dwt)."""
    if csr.rank is None:
        csr = csr_rank_of(idx, xyz.shape[1])
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    O, C = wl.shape[0], 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_bwd_data", "pointconv_bwd_data", xyz, center, feats, idx, wt, wl,
               dy, csr.offsets, csr.rank, bool(need_xyz),
               work=(4 * R * (2 * K * C + 32 * K + O) + 4 * O * 16 * C,
                     4.0 * R * K * C * 16 + 2.0 * R * 16 * C * O))


def pointconv_bwd_weight(xyz, center, feats, idx, wt, dy, o):
    """Weight half of pointconv_bwd -> dwl (O, 16C); reads only its inputs (may run on a
    second stream beside the data half)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    C = 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_bwd_weight", "pointconv_bwd_weight", xyz, center, feats, idx, wt,
               dy, int(o),
               work=(4 * R * (K * C + 16 * K + o) + 4 * o * 16 * C, 2.0 * R * 16 * C * o))



def pointconv_bwd_weight_bias(xyz, center, feats, idx, wt, dy, o):
    """pointconv_bwd_weight plus the bias gradient (column sums of dy) from the same MFMAs
    -> (dwl (O, 16C), dbias (O,)); needs C = 3 + D with C % 8 != 0 (bias_in_weight)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    C = 3 + feats.shape[2]
    R = B * S
    return _op("kdpc_pointconv_bwd_weight", "pointconv_bwd_weight_bias", xyz, center, feats, idx,
               wt, dy, o, work=(4 * R * (K * C + 16 * K + o) + 4 * o * 16 * C,
                                2.0 * R * K * C * 16 + 2.0 * R * 16 * C * o))


def bias_in_weight(feats):
    return BIAS_IN_WEIGHT and (3 + feats.shape[-1]) % 8 != 0


def timing(entry):
    """True when a LaunchTimer brackets `entry` (bench.py's live roofline)."""
    return _timer is not None and entry in _timer.names


# ------------------------------------------------ 3-NN inverse-distance blend
def idw_blend_fwd(ref, qry, vals, idx, warp=False):
    """UpsampleFlow / PointWarping blend: -> (out (B,N,C), w (B,N,3)); see include/kdpc.h."""
    B, S, _ = _gpu(ref, "ref").shape
    N, C = qry.shape[1], vals.shape[2]
    return _op("kdpc_idw_blend_fwd", "idw_blend_fwd", ref, qry, vals, idx, bool(warp),
               work=(4 * B * N * (3 + 3 + 3 * 3 + 3 * C + C + 3), 0))


def idw_blend_bwd_vals(dout, w, csr, S, warp=False):
    """-> dvals (B,S,C) through the CSR of the blend's idx (B,N,3)."""
    return _op("kdpc_idw_blend_bwd_vals", "idw_blend_bwd_vals", _gpu(dout, "dout").contiguous(),
               w, csr.offsets, csr.perm, S, bool(warp))


def idw_blend_bwd_coords(ref, qry, vals, idx, dout, warp=False):
    """-> (drow (B,3N,3) per-neighbour rows of d/d ref, dqry (B,N,3))."""
    return _op("kdpc_idw_blend_bwd_coords", "idw_blend_bwd_coords", _gpu(ref, "ref"), qry,
               vals, idx, dout.contiguous(), bool(warp))


# ------------------------------------------------------------------- fused WeightNet
def weightnet_fwd(xyz, center, idx, params):
    """wt (B,S,K,16) from xyz (B,N,3), center (B,S,3), idx (B,S,K) i32 and the six WeightNet
    tensors params = (W0 (8,3[,1,1]), b0, W1 (8,8), b1, W2 (16,8), b2)."""
    B, N, _ = _gpu(xyz, "xyz").shape
    S, K = idx.shape[1], idx.shape[2]
    return _op("kdpc_weightnet_fwd", "weightnet_fwd", xyz, center, idx, *params,
               work=(B * (12 * N + 12 * S + S * K * (4 + 64)), 2.0 * B * S * K * (24 + 64 + 128)))


def weightnet_bwd(xyz, center, idx, params, dwt, need_rel=False):
    """-> (drel (B,S,K,3) | None, dparams (248,): dW0 | db0 | dW1 | db1 | dW2 | db2)."""
    return _op("kdpc_weightnet_bwd", "weightnet_bwd", _gpu(xyz, "xyz"), center, idx, *params,
               dwt, bool(need_rel))


def weightnet_bwd_rel(xyz, center, idx, params, dwt):
    """drel (B,S,K,3) alone, bit-identical to weightnet_bwd's (the parameter half can then
    run with need_rel=False on another stream)."""
    return _op("kdpc_weightnet_bwd_rel", "weightnet_bwd_rel", _gpu(xyz, "xyz"), center, idx,
               *params, dwt)


# ---------------------------------------------- WeightNet-weighted neighbour sums
def wn_wsum_fwd(dir_, idx, v, params):
    """out (B,N,C) = sum_k WeightNet(dir)[b,q,k,c] * v(b,q,k,c): v (B,N,K,C) for idx None,
    else v[b, idx[b,q,k], c] of v (B,M,C).  params = (W0, b0, W1, b1, W2 (C,8), b2)."""
    B, N, K, _ = _gpu(dir_, "dir").shape
    C = params[4].shape[0]
    vbytes = 4 * (B * N * K * C if idx is None else v.shape[1] * B * C + B * N * K)
    return _op("kdpc_wn_wsum_fwd", "wn_wsum_fwd", dir_, idx, v, *params,
               work=(12 * B * N * K + vbytes + 4 * B * N * C,
                     2.0 * B * N * K * (24 + 64 + 9 * C)))


def wn_wsum_bwd(dir_, idx, v, params, dout):
    """-> dv_rows (B,N,K,C) = w * dout, ddir (B,N,K,3), dparams (104 + 9C)."""
    return _op("kdpc_wn_wsum_bwd", "wn_wsum_bwd", _gpu(dir_, "dir"), idx, v, *params,
               dout.contiguous())


# ------------------------------------------------------- BatchNorm1d + LeakyReLU (rows)
def batchnorm_lrelu_fwd(x2, weight, bias, eps, momentum, slope, run_mean, run_var):
    """Train mode over x2 (R, C): -> (y, mean, invstd); running stats updated in place."""
    R, C = _gpu(x2, "x").shape
    return _op("kdpc_batchnorm_lrelu_fwd", "batchnorm_lrelu_fwd", x2, weight, bias, float(eps),
               float(momentum), float(slope), run_mean, run_var, work=(12 * R * C, 0))


def batchnorm_lrelu_apply(x2, mean, invstd, weight, bias, slope):
    return _op("kdpc_batchnorm_lrelu_apply", "batchnorm_lrelu_apply", _gpu(x2, "x"), mean,
               invstd, weight, bias, float(slope))


def batchnorm_lrelu_bwd(dy, y, x2, weight, mean, invstd, slope):
    """-> (dx, dweight, dbias)."""
    R, C = _gpu(x2, "x").shape
    return _op("kdpc_batchnorm_lrelu_bwd", "batchnorm_lrelu_bwd", dy, y, x2, weight, mean,
               invstd, float(slope), work=(20 * R * C, 0))


@functools.lru_cache(maxsize=None)
def dense_tn_small_supported(r, o, i):
    return load_library().kdpc_dense_tn_small_workspace_bytes(r, o, i) > 0


def dense_tn_small(a, b):
    """a (R,O), b (R,I) -> a^T b (O,I) for tiny O*I (see include/kdpc.h)."""
    R, O = _gpu(a, "a").shape
    I = b.shape[1]
    return _op("kdpc_dense_tn_small", "dense_tn_small", a.contiguous(), b.contiguous(),
               work=(4 * R * (O + I) + 4 * O * I, 2.0 * R * O * I))


def dense_small(x2, m, bias=None):
    """x2 (R,K) @ m (K,N) [+ bias] for min(K, N) <= 4 (see include/kdpc.h)."""
    R, K = _gpu(x2, "x").shape
    N = m.shape[1]
    return _op("kdpc_dense_small", "dense_small", x2.contiguous(), m.contiguous(), bias,
               work=(4 * (R * K + R * N + K * N), 2.0 * R * K * N))


def dense_small_out(x2, m, bias, y2):
    """dense_small into y2 (R,N), a contiguous view of a caller-owned output."""
    R, K = _gpu(x2, "x").shape
    N = m.shape[1]
    _op("kdpc_dense_small", "dense_small_out", x2.contiguous(), m.contiguous(), bias, y2,
        work=(4 * (R * K + R * N + K * N), 2.0 * R * K * N))


def neg_sum_k(x):
    """x (..., K, C) -> -x.sum(-2) (..., C), ascending-K order, one launch."""
    return _op("kdpc_neg_sum_k", "neg_sum_k", _gpu(x, "x").contiguous())


# torch's fused Adam over the flat buffers of distill.GraphedStep, as one full-chip launch
# (csrc/adam.hip); ADAM_MODE: how the update is evaluated (bit 0 contracted double expressions,
# bit 1 fast f32 division / sqrt): the form tests/test_gpu_adam.py finds bit-identical to
# torch's fused Adam
ADAM_MODE = 1


def adam_step(param, grad, exp_avg, exp_avg_sq, lr, step, beta1, beta2, eps, weight_decay,
              maximize=False, mode=None):
    """In-place Adam on flat f32 buffers (n % 4 == 0, 16-byte aligned); lr / step: device
    scalars, step already incremented."""
    c = ADAM_MODE if mode is None else int(mode)
    n = _gpu(param, "param").numel()
    _op("kdpc_adam_step", "adam_step", param, grad, exp_avg, exp_avg_sq, lr, step,
        float(beta1), float(beta2), float(eps), float(weight_decay), bool(maximize), c,
        work=(28.0 * n, 0.0))


def copy_segments(dst, src):
    """dst[i].copy_(src[i]) for same-size contiguous tensors, ceil(n/128) launches."""
    dst, src = list(dst), list(src)
    _op("kdpc_copy_segments", "copy_segments", dst, src,
        work=(2.0 * sum(s.numel() * s.element_size() for s in src), 0.0))


def colsum(x2):
    """Column sums of a row-major (R, L) tensor, deterministic fixed-order: -> (L,)."""
    return _op("kdpc_colsum", "colsum", _gpu(x2, "src"))
