"""Drop-in for the reference's pybind module `pointnet2_cuda` (pointnet2_api.cpp:10-24).

The nine `*_wrapper` functions keep the reference's argument lists and in-place contract
(caller-allocated GPU tensors), so the reference's own pointnet2_utils.py runs unchanged on
top of them.  Each forwards to the matching C-ABI entry point in include/kdpc.h.
Deterministic backward: *_grad_wrapper overwrites grad_points (the reference accumulated
into a caller-zeroed buffer with atomics; the result for a zeroed buffer is the same sum);
their scratch comes from the torch caching allocator (the C ABI's *_grad_ws entry points).
"""
import kdpc_native as _nat


def _p(t, dtype, name):
    return _nat._dev(t, dtype, name)


def _f(t, name):
    import torch
    return _p(t, torch.float32, name)


def _i(t, name):
    import torch
    return _p(t, torch.int32, name)


def ball_query_wrapper(b, n, m, radius, nsample, new_xyz, xyz, idx):
    _nat._call("kdpc_ball_query", b, n, m, float(radius), nsample, _f(new_xyz, "new_xyz"),
               _f(xyz, "xyz"), _i(idx, "idx"), _nat._stream(xyz))
    return 1


def group_points_wrapper(b, c, n, npoints, nsample, points, idx, out):
    _nat._call("kdpc_group_points", b, c, n, npoints, nsample, _f(points, "points"),
               _i(idx, "idx"), _f(out, "out"), _nat._stream(points))
    return 1


def _ws(n, p, like):
    """Scratch of a *_grad_ws call from the torch caching allocator (stream-ordered with the
    op, graph-capture safe)."""
    import torch
    nbytes = _nat.load_library().kdpc_grad_workspace_bytes(n[0], n[1], p)
    ws = torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device=like.device)
    return ws.data_ptr(), nbytes


def group_points_grad_wrapper(b, c, n, npoints, nsample, grad_out, idx, grad_points):
    ws, nb = _ws((b, n), npoints * nsample, grad_out)
    _nat._call("kdpc_group_points_grad_ws", b, c, n, npoints, nsample, _f(grad_out, "grad_out"),
               _i(idx, "idx"), _f(grad_points, "grad_points"), ws, nb, _nat._stream(grad_out))
    return 1


def gather_points_wrapper(b, c, n, npoints, points, idx, out):
    _nat._call("kdpc_gather_points", b, c, n, npoints, _f(points, "points"), _i(idx, "idx"),
               _f(out, "out"), _nat._stream(points))
    return 1


def gather_points_grad_wrapper(b, c, n, npoints, grad_out, idx, grad_points):
    ws, nb = _ws((b, n), npoints, grad_out)
    _nat._call("kdpc_gather_points_grad_ws", b, c, n, npoints, _f(grad_out, "grad_out"),
               _i(idx, "idx"), _f(grad_points, "grad_points"), ws, nb, _nat._stream(grad_out))
    return 1


def furthest_point_sampling_wrapper(b, n, m, points, temp, idx):
    _nat._call("kdpc_furthest_point_sampling", b, n, m, _f(points, "points"), _f(temp, "temp"),
               _i(idx, "idx"), _nat._stream(points))
    return 1


def three_nn_wrapper(b, n, m, unknown, known, dist2, idx):
    _nat._call("kdpc_three_nn", b, n, m, _f(unknown, "unknown"), _f(known, "known"),
               _f(dist2, "dist2"), _i(idx, "idx"), _nat._stream(unknown))


def three_interpolate_wrapper(b, c, m, n, points, idx, weight, out):
    _nat._call("kdpc_three_interpolate", b, c, m, n, _f(points, "points"), _i(idx, "idx"),
               _f(weight, "weight"), _f(out, "out"), _nat._stream(points))


def three_interpolate_grad_wrapper(b, c, n, m, grad_out, idx, weight, grad_points):
    ws, nb = _ws((b, m), 3 * n, grad_out)
    _nat._call("kdpc_three_interpolate_grad_ws", b, c, n, m, _f(grad_out, "grad_out"),
               _i(idx, "idx"), _f(weight, "weight"), _f(grad_points, "grad_points"), ws, nb,
               _nat._stream(grad_out))
