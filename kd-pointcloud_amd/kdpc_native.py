"""ctypes binding of libkdpc_hip.so (the C ABI in include/kdpc.h) for torch-ROCm tensors.

Every op here runs the gfx950 HIP kernels on the tensors' device and the current torch
stream.  There is no CPU path: a missing library, a CPU tensor or a wrong dtype raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KDPC_LIB", os.path.join(_HERE, "lib", "libkdpc_hip.so"))

_c_int, _c_float, _c_size, _vp = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p

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
    "kdpc_group_rows": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "kdpc_csr_workspace_bytes": [_c_int, _c_int, _c_int],
    "kdpc_csr_build": [_c_int, _c_int, _c_int, _vp, _vp, _c_size, _vp, _vp, _vp],
    "kdpc_group_rows_grad_csr": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_csr_sum_channels": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "kdpc_three_interpolate_grad_csr": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp,
                                        _vp, _vp],
    "kdpc_cost_volume_fwd": [_c_int] * 6 + [_vp] * 12,
    "kdpc_pointconv_contract_fwd": [_c_int] * 5 + [_vp] * 7,
    "kdpc_pointconv_contract_bwd": [_c_int] * 5 + [_vp] * 10,
    "kdpc_cost_volume_bwd_workspace_bytes": [_c_int] * 4,
    "kdpc_cost_volume_bwd": [_c_int] * 6 + [_vp] * 16 + [_c_size, _vp, _vp],
    "kdpc_pointconv_supported": [_c_int] * 3,
    "kdpc_pointconv_fwd_workspace_bytes": [_c_int] * 5,
    "kdpc_pointconv_fwd": [_c_int] * 6 + [_vp] * 9 + [_c_size, _vp],
    "kdpc_pointconv_bwd_workspace_bytes": [_c_int] * 5,
    "kdpc_pointconv_bwd": [_c_int] * 6 + [_vp] * 15 + [_c_size, _vp],
    "kdpc_batchnorm_workspace_bytes": [_c_int, _c_int],
    "kdpc_batchnorm_lrelu_fwd": [_c_int, _c_int] + [_vp] * 3 + [_c_float] * 3 + [_vp] * 6
                                + [_c_size, _vp],
    "kdpc_batchnorm_lrelu_apply": [_c_int, _c_int] + [_vp] * 5 + [_c_float, _vp, _vp],
    "kdpc_batchnorm_lrelu_bwd": [_c_int, _c_int] + [_vp] * 6 + [_c_float] + [_vp] * 4
                                + [_c_size, _vp],
    "kdpc_colsum_workspace_bytes": [_c_int, _c_int],
    "kdpc_colsum": [_c_int, _c_int, _vp, _vp, _vp, _c_size, _vp],
    "kdpc_weightnet_param_count": [],
    "kdpc_weightnet_fwd": [_c_int] * 4 + [_vp] * 11,
    "kdpc_weightnet_bwd_workspace_bytes": [],
    "kdpc_weightnet_bwd": [_c_int] * 4 + [_vp] * 13 + [_c_size, _vp],
}
_RESTYPES = {"kdpc_build_id": ctypes.c_char_p, "kdpc_grad_workspace_bytes": _c_size,
             "kdpc_csr_workspace_bytes": _c_size, "kdpc_cost_volume_bwd_workspace_bytes": _c_size,
             "kdpc_pointconv_fwd_workspace_bytes": _c_size,
             "kdpc_pointconv_bwd_workspace_bytes": _c_size,
             "kdpc_weightnet_bwd_workspace_bytes": _c_size,
             "kdpc_batchnorm_workspace_bytes": _c_size,
             "kdpc_colsum_workspace_bytes": _c_size, "kdpc_knn_workspace_bytes": _c_size}

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
    got = lib.kdpc_build_id().decode()
    if got != want:
        raise KdpcError(f"{path} was built from other sources (build id {got[:12]}, sources "
                        f"{want[:12]}); rebuild with `python kd-pointcloud_amd/build_native.py`")


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

    def __init__(self, names):
        self.names = set(names)
        self.records = []  # (name, start_event, end_event, bytes, flops)

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
    """Invoke a C entry point; `work` = (algorithmic bytes, flops) for the launch timer."""
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


# ------------------------------------------------------------------------------ ops
def furthest_point_sampling(xyz, npoint, temp=None):
    """xyz (B,N,3) f32 -> idx (B,npoint) i32.  temp: optional (B,N) scratch (1e10-filled)."""
    B, N, _ = xyz.shape
    idx = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
    if temp is None:
        temp = torch.full((B, N), 1e10, dtype=torch.float32, device=xyz.device)
    _call("kdpc_furthest_point_sampling", B, N, npoint, _dev(xyz, torch.float32, "xyz"),
          _dev(temp, torch.float32, "temp"), _dev(idx, torch.int32, "idx"), _stream(xyz),
          work=(B * (12 * N + 8 * N + 4 * npoint), B * N * npoint * 8))
    return idx


def gather_points(points, idx):
    """points (B,C,N), idx (B,M) i32 -> (B,C,M)."""
    B, C, N = points.shape
    M = idx.shape[1]
    out = torch.empty((B, C, M), dtype=torch.float32, device=points.device)
    _call("kdpc_gather_points", B, C, N, M, _dev(points, torch.float32, "points"),
          _dev(idx, torch.int32, "idx"), _dev(out, torch.float32, "out"), _stream(points))
    return out


def ball_query(radius, nsample, xyz, new_xyz):
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    idx = torch.empty((B, M, nsample), dtype=torch.int32, device=xyz.device)
    _call("kdpc_ball_query", B, N, M, float(radius), int(nsample),
          _dev(new_xyz, torch.float32, "new_xyz"), _dev(xyz, torch.float32, "xyz"),
          _dev(idx, torch.int32, "idx"), _stream(xyz))
    return idx


def group_points(points, idx):
    """points (B,C,N), idx (B,S,K) i32 -> (B,C,S,K)."""
    B, C, N = points.shape
    _, S, K = idx.shape
    out = torch.empty((B, C, S, K), dtype=torch.float32, device=points.device)
    # SURVEY §8d algorithmic bytes: B*(4CN + 4SK + 4CSK)
    _call("kdpc_group_points", B, C, N, S, K, _dev(points, torch.float32, "points"),
          _dev(idx, torch.int32, "idx"), _dev(out, torch.float32, "out"), _stream(points),
          work=(B * (4 * C * N + 4 * S * K + 4 * C * S * K), 0))
    return out


def three_nn(unknown, known):
    """-> (dist2 (B,N,3) squared, idx (B,N,3) i32)."""
    B, N, _ = unknown.shape
    M = known.shape[1]
    dist2 = torch.empty((B, N, 3), dtype=torch.float32, device=unknown.device)
    idx = torch.empty((B, N, 3), dtype=torch.int32, device=unknown.device)
    _call("kdpc_three_nn", B, N, M, _dev(unknown, torch.float32, "unknown"),
          _dev(known, torch.float32, "known"), _dev(dist2, torch.float32, "dist2"),
          _dev(idx, torch.int32, "idx"), _stream(unknown))
    return dist2, idx


def three_interpolate(points, idx, weight):
    B, C, M = points.shape
    N = idx.shape[1]
    out = torch.empty((B, C, N), dtype=torch.float32, device=points.device)
    _call("kdpc_three_interpolate", B, C, M, N, _dev(points, torch.float32, "points"),
          _dev(idx, torch.int32, "idx"), _dev(weight, torch.float32, "weight"),
          _dev(out, torch.float32, "out"), _stream(points))
    return out


def knn_point(nsample, xyz, new_xyz, return_dist=False, seeded=True):
    """xyz (B,N,3) refs, new_xyz (B,S,3) queries -> idx (B,S,K) i32 ascending (dist, idx).
    seeded: allow the seeded-threshold scan where it pays (identical results; False forces
    the unseeded scan, for tests)."""
    B, N, _ = xyz.shape
    S = new_xyz.shape[1]
    if nsample > N:
        raise ValueError(f"knn_point: nsample={nsample} > number of points {N}")
    idx = torch.empty((B, S, nsample), dtype=torch.int32, device=xyz.device)
    dist = torch.empty((B, S, nsample), dtype=torch.float32, device=xyz.device) if return_dist else None
    ws_bytes = load_library().kdpc_knn_workspace_bytes(B, N, S) if seeded else 0
    ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=xyz.device) if ws_bytes else None
    _call("kdpc_knn_point_ws", B, N, S, int(nsample), _dev(xyz, torch.float32, "xyz"),
          _dev(new_xyz, torch.float32, "new_xyz"), _dev(idx, torch.int32, "idx"),
          _dev(dist, torch.float32, "dist") if dist is not None else None,
          ws.data_ptr() if ws is not None else None, ws_bytes, _stream(xyz),
          work=(B * (12 * N + 12 * S + 4 * S * nsample * (2 if return_dist else 1)),
                B * S * N * 8))
    return (idx, dist) if return_dist else idx


def group_rows(points, idx):
    """points (B,N,C), idx (B,P) i32 -> (B,P,C) (point-major row gather)."""
    B, N, C = points.shape
    P = idx.shape[1]
    out = torch.empty((B, P, C), dtype=torch.float32, device=points.device)
    # algorithmic bytes: table read once + idx read + rows written
    _call("kdpc_group_rows", B, N, C, P, _dev(points, torch.float32, "points"),
          _dev(idx, torch.int32, "idx"), _dev(out, torch.float32, "out"), _stream(points),
          work=(B * (4 * N * C + 4 * P + 4 * P * C), 0))
    return out


class Csr:
    """Inverted index of an int32 index tensor (B,P) over a key space of n values."""
    __slots__ = ("offsets", "perm", "n", "p")

    def __init__(self, idx2d, n):
        B, P = idx2d.shape
        lib = load_library()
        ws_bytes = lib.kdpc_csr_workspace_bytes(B, n, P)
        if ws_bytes == 0:
            raise KdpcError("kdpc_csr_workspace_bytes returned 0 (invalid sizes?)")
        dev = idx2d.device
        ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=dev)
        self.offsets = torch.empty((B * n + 1,), dtype=torch.int32, device=dev)
        self.perm = torch.empty((B * P,), dtype=torch.int32, device=dev)
        self.n, self.p = n, P
        _call("kdpc_csr_build", B, n, P, _dev(idx2d, torch.int32, "idx"), ws.data_ptr(), ws_bytes,
              self.offsets.data_ptr(), self.perm.data_ptr(), _stream(idx2d))


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
    else:
        csr = Csr(idx.reshape(idx.shape[0], -1), n)
    try:
        idx._kdpc_csr = csr
    except AttributeError:
        pass
    return csr


def group_rows_grad(grad_out, csr, B, N, C):
    """grad_out (B,P,C) -> (B,N,C) deterministic scatter-add through csr."""
    grad_out = grad_out.contiguous()
    out = torch.empty((B, N, C), dtype=torch.float32, device=grad_out.device)
    P = grad_out.shape[1]
    _call("kdpc_group_rows_grad_csr", B, N, C, _dev(grad_out, torch.float32, "grad_out"),
          csr.offsets.data_ptr(), csr.perm.data_ptr(), _dev(out, torch.float32, "grad_points"),
          _stream(grad_out), work=(B * (4 * P * C + 4 * P + 4 * N + 4 * N * C), 0))
    return out


def csr_sum_channels(src, csr, B, C, N):
    """src (B,C,P) -> (B,C,N): the backward of gather_points/group_points."""
    src = src.contiguous()
    P = src.numel() // max(1, B * C)
    out = torch.empty((B, C, N), dtype=torch.float32, device=src.device)
    _call("kdpc_csr_sum_channels", B, C, N, P, _dev(src, torch.float32, "src"),
          csr.offsets.data_ptr(), csr.perm.data_ptr(), _dev(out, torch.float32, "dst"),
          _stream(src))
    return out


def three_interpolate_grad(grad_out, idx, weight, m):
    """grad_out (B,C,N) -> (B,C,M) deterministic."""
    grad_out = grad_out.contiguous()
    B, C, N = grad_out.shape
    csr = csr_of(idx, m)
    out = torch.empty((B, C, m), dtype=torch.float32, device=grad_out.device)
    _call("kdpc_three_interpolate_grad_csr", B, C, N, m, _dev(grad_out, torch.float32, "grad_out"),
          _dev(weight, torch.float32, "weight"), csr.offsets.data_ptr(), csr.perm.data_ptr(),
          _dev(out, torch.float32, "grad_points"), _stream(grad_out))
    return out


# ------------------------------------------------------------------ fused cost volume
def cost_volume_supported(din, dout, k):
    return din in (32, 64) and dout in (32, 64) and 1 <= k <= 32


def cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1):
    """-> out (B,N1,Dout) f32, amax (B,N1,Dout) u8.  See include/kdpc.h."""
    B, N1, _ = x1.shape
    N2 = x2.shape[1]
    K = idx.shape[2]
    din, dout = p1.shape[2], w1.shape[0]
    out = torch.empty((B, N1, dout), dtype=torch.float32, device=x1.device)
    amax = torch.empty((B, N1, dout), dtype=torch.uint8, device=x1.device)
    f = torch.float32
    _call("kdpc_cost_volume_fwd", B, N1, N2, K, din, dout, _dev(x1, f, "x1"), _dev(x2, f, "x2"),
          _dev(idx, torch.int32, "idx"), _dev(p1, f, "p1"), _dev(p2, f, "p2"),
          _dev(wpos, f, "wpos"), _dev(bpos, f, "bpos"), _dev(w1, f, "w1"), _dev(b1, f, "b1"),
          _dev(out, f, "out"), _dev(amax, torch.uint8, "amax"), _stream(x1),
          work=(4 * B * N1 * (3 + K + din + K * din + 2 * dout) + B * N1 * dout,
                2.0 * B * N1 * K * din * dout))
    return out, amax


def cost_volume_bwd(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout):
    """-> dp1 (B,N1,Din), dp2_rows (B,N1,K,Din), dx1 (B,N1,3), ddir_rows (B,N1,K,3), dparams."""
    B, N1, _ = x1.shape
    N2 = x2.shape[1]
    K = idx.shape[2]
    din, dout = p1.shape[2], w1.shape[0]
    dev = x1.device
    f = torch.float32
    dp1 = torch.empty((B, N1, din), dtype=f, device=dev)
    dp2_rows = torch.empty((B, N1, K, din), dtype=f, device=dev)
    dx1 = torch.empty((B, N1, 3), dtype=f, device=dev)
    ddir_rows = torch.empty((B, N1, K, 3), dtype=f, device=dev)
    dparams = torch.empty((dout * din + dout + 4 * din,), dtype=f, device=dev)
    lib = load_library()
    ws_bytes = lib.kdpc_cost_volume_bwd_workspace_bytes(B, N1, din, dout)
    ws = torch.empty((max(ws_bytes, 4),), dtype=torch.uint8, device=dev)
    _call("kdpc_cost_volume_bwd", B, N1, N2, K, din, dout, _dev(x1, f, "x1"), _dev(x2, f, "x2"),
          _dev(idx, torch.int32, "idx"), _dev(p1, f, "p1"), _dev(p2, f, "p2"),
          _dev(wpos, f, "wpos"), _dev(bpos, f, "bpos"), _dev(w1, f, "w1"), _dev(out, f, "out"),
          _dev(amax, torch.uint8, "amax"), _dev(gout, f, "dout"), _dev(dp1, f, "dp1"),
          _dev(dp2_rows, f, "dp2_rows"), _dev(dx1, f, "dx1"), _dev(ddir_rows, f, "ddir_rows"),
          ws.data_ptr(), ws_bytes, _dev(dparams, f, "dparams"), _stream(x1))
    return dp1, dp2_rows, dx1, ddir_rows, dparams


# ------------------------------------------------------------------ wide cost volume
def cost_volume_wide_supported(din, dout, k):
    return bool(load_library().kdpc_cost_volume_wide_supported(din, dout, k))


def cost_volume_wide_h0(x1, x2, idx, p1, p2, wpos, bpos):
    """-> h0 (B,N1,K,Din) = LeakyReLU(P2[idx] + P1 + Wpos dir + bpos)."""
    B, N1, _ = x1.shape
    N2, K, din = x2.shape[1], idx.shape[2], p1.shape[2]
    f = torch.float32
    h0 = torch.empty((B, N1, K, din), dtype=f, device=x1.device)
    _call("kdpc_cost_volume_wide_h0", B, N1, N2, K, din, _dev(x1, f, "x1"), _dev(x2, f, "x2"),
          _dev(idx, torch.int32, "idx"), _dev(p1, f, "p1"), _dev(p2, f, "p2"),
          _dev(wpos, f, "wpos"), _dev(bpos, f, "bpos"), _dev(h0, f, "h0"), _stream(x1),
          work=(4 * B * N1 * (K * (1 + 2 * din + 3) + din + 3), 10.0 * B * N1 * K * din))
    return h0


def cost_volume_wide_max(z1, B, N1, K, dout):
    """z1 (B*N1*K, Dout) -> out (B,N1,Dout), amax (B,N1,Dout) u8."""
    f = torch.float32
    out = torch.empty((B, N1, dout), dtype=f, device=z1.device)
    amax = torch.empty((B, N1, dout), dtype=torch.uint8, device=z1.device)
    _call("kdpc_cost_volume_wide_max", B, N1, K, dout, _dev(z1, f, "z1"), _dev(out, f, "out"),
          _dev(amax, torch.uint8, "amax"), _stream(z1))
    return out, amax


def cost_volume_wide_max_bwd(gout, out, amax, K):
    """-> dz1 (B*N1*K, Dout) dense, gsc (B*N1, Dout)."""
    B, N1, dout = out.shape
    f = torch.float32
    dz1 = torch.empty((B * N1 * K, dout), dtype=f, device=out.device)
    gsc = torch.empty((B * N1, dout), dtype=f, device=out.device)
    _call("kdpc_cost_volume_wide_max_bwd", B, N1, K, dout, _dev(gout, f, "gout"),
          _dev(out, f, "out"), _dev(amax, torch.uint8, "amax"), _dev(dz1, f, "dz1"),
          _dev(gsc, f, "gsc"), _stream(out))
    return dz1, gsc


def cost_volume_wide_h0_bwd(x1, x2, idx, h0, dz):
    """dz (B*N1*K, Din) dh0 -> dz0 in place; -> dp1 (B,N1,Din), dWpos (Din,3)."""
    B, N1, _ = x1.shape
    N2, K, din = x2.shape[1], idx.shape[2], h0.shape[-1]
    f = torch.float32
    lib = load_library()
    rows = lib.kdpc_cost_volume_wide_slab_rows()
    slab = torch.empty((rows, din * 3), dtype=f, device=x1.device)
    dp1 = torch.empty((B, N1, din), dtype=f, device=x1.device)
    _call("kdpc_cost_volume_wide_h0_bwd", B, N1, N2, K, din, _dev(x1, f, "x1"), _dev(x2, f, "x2"),
          _dev(idx, torch.int32, "idx"), _dev(h0, f, "h0"), _dev(dz, f, "dz"),
          _dev(dp1, f, "dp1"), _dev(slab, f, "slab"), _stream(x1))
    return dp1, colsum(slab).view(din, 3)


# ------------------------------------------------------------------ PointConv contraction
def pointconv_contract_fwd(xyz, center, feats, idx, wt):
    """-> A (B,S,16*(3+D)), c-major (the reference's .view(B,S,-1) of (B,S,C,16))."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    D = feats.shape[2]
    C = 3 + D
    out = torch.empty((B, S, 16 * C), dtype=torch.float32, device=xyz.device)
    f = torch.float32
    _call("kdpc_pointconv_contract_fwd", B, N, S, K, D, _dev(xyz, f, "xyz"),
          _dev(center, f, "center"), _dev(feats, f, "feats"), _dev(idx, torch.int32, "idx"),
          _dev(wt, f, "wt"), _dev(out, f, "out"), _stream(xyz),
          work=(4 * B * S * (K + K * C + 16 * K + 16 * C), 2.0 * B * S * K * C * 16))
    return out


def pointconv_contract_bwd(xyz, center, feats, idx, wt, dout):
    """-> dg_rows (B,S,K,3+D), dwt (B,S,K,16), dcenter (B,S,3)."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    D = feats.shape[2]
    C = 3 + D
    dev = xyz.device
    f = torch.float32
    dg_rows = torch.empty((B, S, K, C), dtype=f, device=dev)
    dwt = torch.empty((B, S, K, 16), dtype=f, device=dev)
    dcenter = torch.empty((B, S, 3), dtype=f, device=dev)
    _call("kdpc_pointconv_contract_bwd", B, N, S, K, D, _dev(xyz, f, "xyz"),
          _dev(center, f, "center"), _dev(feats, f, "feats"), _dev(idx, torch.int32, "idx"),
          _dev(wt, f, "wt"), _dev(dout, f, "dout"), _dev(dg_rows, f, "dg_rows"),
          _dev(dwt, f, "dwt"), _dev(dcenter, f, "dcenter"), _stream(xyz))
    return dg_rows, dwt, dcenter


# ------------------------------------------------------------------ fused PointConv layer
def pointconv_supported(k, d, o):
    return bool(load_library().kdpc_pointconv_supported(k, d, o))


def _workspace(nbytes, device):
    return torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device=device)


def pointconv_fwd(xyz, center, feats, idx, wt, wl, bias):
    """Fused gather + contraction + Linear: -> y (B,S,O) = A wl^T + bias, A never stored.
    xyz (B,N,3), center (B,S,3), feats (B,N,D), idx (B,S,K) i32, wt (B,S,K,16), wl (O,16C)."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    D = feats.shape[2]
    O = wl.shape[0]
    C = 3 + D
    f = torch.float32
    lib = load_library()
    ws_bytes = lib.kdpc_pointconv_fwd_workspace_bytes(B, S, K, D, O)
    ws = _workspace(ws_bytes, xyz.device)
    y = torch.empty((B, S, O), dtype=f, device=xyz.device)
    R = B * S
    _call("kdpc_pointconv_fwd", B, N, S, K, D, O, _dev(xyz, f, "xyz"), _dev(center, f, "center"),
          _dev(feats, f, "feats"), _dev(idx, torch.int32, "idx"), _dev(wt, f, "wt"),
          _dev(wl, f, "wl"), _dev(bias, f, "bias"), _dev(y, f, "y"), ws.data_ptr(), ws_bytes,
          _stream(xyz),
          work=(4 * R * (K + K * C + 16 * K + O) + 4 * O * 16 * C,
                2.0 * R * K * C * 16 + 2.0 * R * 16 * C * O))
    return y


def pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=True):
    """Backward of pointconv_fwd for dy (B,S,O) -> (dxyz|None, dfeats, dcenter, dwt, dwl)."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    D = feats.shape[2]
    O = wl.shape[0]
    C = 3 + D
    f = torch.float32
    dev = xyz.device
    lib = load_library()
    ws_bytes = lib.kdpc_pointconv_bwd_workspace_bytes(B, S, K, D, O)
    if ws_bytes == 0:
        raise KdpcError("kdpc_pointconv_bwd_workspace_bytes returned 0 (invalid sizes?)")
    ws = _workspace(ws_bytes, dev)
    dxyz = torch.empty((B, N, 3), dtype=f, device=dev) if need_xyz else None
    dfeats = torch.empty((B, N, D), dtype=f, device=dev)
    dcenter = torch.empty((B, S, 3), dtype=f, device=dev)
    dwt = torch.empty((B, S, K, 16), dtype=f, device=dev)
    dwl = torch.empty((O, 16 * C), dtype=f, device=dev)
    R = B * S
    _call("kdpc_pointconv_bwd", B, N, S, K, D, O, _dev(xyz, f, "xyz"), _dev(center, f, "center"),
          _dev(feats, f, "feats"), _dev(idx, torch.int32, "idx"), _dev(wt, f, "wt"),
          _dev(wl, f, "wl"), _dev(dy, f, "dy"), csr.offsets.data_ptr(), csr.perm.data_ptr(),
          dxyz.data_ptr() if need_xyz else None, _dev(dfeats, f, "dfeats"),
          _dev(dcenter, f, "dcenter"), _dev(dwt, f, "dwt"), _dev(dwl, f, "dwl"), ws.data_ptr(),
          ws_bytes, _stream(xyz),
          work=(4 * R * (2 * K * C + 32 * K + 2 * O) + 8 * O * 16 * C,
                4.0 * R * K * C * 16 + 4.0 * R * 16 * C * O))
    return dxyz, dfeats, dcenter, dwt, dwl


# ------------------------------------------------------------------- fused WeightNet
def weightnet_fwd(xyz, center, idx, params):
    """wt (B,S,K,16) from xyz (B,N,3), center (B,S,3), idx (B,S,K) i32 and the six WeightNet
    tensors params = (W0 (8,3[,1,1]), b0, W1 (8,8), b1, W2 (16,8), b2)."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    f = torch.float32
    wt = torch.empty((B, S, K, 16), dtype=f, device=xyz.device)
    ptrs = [_dev(p, f, f"weightnet param {i}") for i, p in enumerate(params)]
    _call("kdpc_weightnet_fwd", B, N, S, K, _dev(xyz, f, "xyz"), _dev(center, f, "center"),
          _dev(idx, torch.int32, "idx"), *ptrs, _dev(wt, f, "wt"), _stream(xyz),
          work=(B * (12 * N + 12 * S + S * K * (4 + 64)), 2.0 * B * S * K * (24 + 64 + 128)))
    return wt


def weightnet_bwd(xyz, center, idx, params, dwt, need_rel=False):
    """-> (drel (B,S,K,3) | None, dparams (248,): dW0 | db0 | dW1 | db1 | dW2 | db2)."""
    B, N, _ = xyz.shape
    S, K = idx.shape[1], idx.shape[2]
    f = torch.float32
    dev = xyz.device
    lib = load_library()
    ws_bytes = lib.kdpc_weightnet_bwd_workspace_bytes()
    ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=dev)
    dparams = torch.empty((lib.kdpc_weightnet_param_count(),), dtype=f, device=dev)
    drel = torch.empty((B, S, K, 3), dtype=f, device=dev) if need_rel else None
    ptrs = [_dev(p, f, f"weightnet param {i}") for i, p in enumerate(params)]
    _call("kdpc_weightnet_bwd", B, N, S, K, _dev(xyz, f, "xyz"), _dev(center, f, "center"),
          _dev(idx, torch.int32, "idx"), *ptrs, _dev(dwt, f, "dwt"),
          drel.data_ptr() if need_rel else None, dparams.data_ptr(), ws.data_ptr(), ws_bytes,
          _stream(xyz))
    return drel, dparams


# ------------------------------------------------------- BatchNorm1d + LeakyReLU (rows)
def batchnorm_lrelu_fwd(x2, weight, bias, eps, momentum, slope, run_mean, run_var):
    """Train mode over x2 (R, C): -> (y, mean, invstd); running stats updated in place."""
    R, C = x2.shape
    f = torch.float32
    dev = x2.device
    lib = load_library()
    ws = _workspace(lib.kdpc_batchnorm_workspace_bytes(R, C), dev)
    y = torch.empty_like(x2)
    mean = torch.empty((C,), dtype=f, device=dev)
    invstd = torch.empty((C,), dtype=f, device=dev)
    _call("kdpc_batchnorm_lrelu_fwd", R, C, _dev(x2, f, "x"), _dev(weight, f, "weight"),
          _dev(bias, f, "bias"), float(eps), float(momentum), float(slope),
          None if run_mean is None else _dev(run_mean, f, "running_mean"),
          None if run_var is None else _dev(run_var, f, "running_var"),
          mean.data_ptr(), invstd.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel(),
          _stream(x2), work=(12 * R * C, 0))
    return y, mean, invstd


def batchnorm_lrelu_apply(x2, mean, invstd, weight, bias, slope):
    R, C = x2.shape
    f = torch.float32
    y = torch.empty_like(x2)
    _call("kdpc_batchnorm_lrelu_apply", R, C, _dev(x2, f, "x"), _dev(mean, f, "mean"),
          _dev(invstd, f, "invstd"), _dev(weight, f, "weight"), _dev(bias, f, "bias"),
          float(slope), y.data_ptr(), _stream(x2))
    return y


def batchnorm_lrelu_bwd(dy, y, x2, weight, mean, invstd, slope):
    """-> (dx, dweight, dbias)."""
    R, C = x2.shape
    f = torch.float32
    dev = x2.device
    lib = load_library()
    ws = _workspace(lib.kdpc_batchnorm_workspace_bytes(R, C), dev)
    dx = torch.empty_like(x2)
    dw = torch.empty((C,), dtype=f, device=dev)
    db = torch.empty((C,), dtype=f, device=dev)
    _call("kdpc_batchnorm_lrelu_bwd", R, C, _dev(dy, f, "dy"), _dev(y, f, "y"), _dev(x2, f, "x"),
          _dev(weight, f, "weight"), _dev(mean, f, "mean"), _dev(invstd, f, "invstd"),
          float(slope), dx.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(),
          _stream(x2), work=(20 * R * C, 0))
    return dx, dw, db


def colsum(x2):
    """Column sums of a row-major (R, L) tensor, deterministic fixed-order: -> (L,)."""
    R, L = x2.shape
    f = torch.float32
    lib = load_library()
    nb = lib.kdpc_colsum_workspace_bytes(R, L)
    ws = _workspace(nb, x2.device)
    out = torch.empty((L,), dtype=f, device=x2.device)
    _call("kdpc_colsum", R, L, _dev(x2, f, "src"), out.data_ptr(), ws.data_ptr(), nb,
          _stream(x2))
    return out
