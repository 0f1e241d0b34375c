"""Drop-in for the reference's pybind module `pointnet2_cuda` (pointnet2_api.cpp:10-24).

The nine `*_wrapper` functions keep the reference's argument lists and in-place contract
(caller-allocated GPU tensors), so the reference's own pointnet2_utils.py runs unchanged on
top of them.  Each is the torch operator of the same name, torch.ops.kdpc.<name>
(torch_ops/kdpc_torch_ops.cpp), which checks its tensors and calls the matching C-ABI entry
point of include/kdpc.h on the current stream.  Deterministic backward: *_grad_wrapper
overwrites grad_points (the reference accumulated into a caller-zeroed buffer with atomics;
the result for a zeroed buffer is the same sum); its scratch comes from the torch caching
allocator.
"""
import kdpc_native as _nat


def _ops():
    return _nat.load_ops()


def ball_query_wrapper(b, n, m, radius, nsample, new_xyz, xyz, idx):
    return _ops().ball_query_wrapper(b, n, m, float(radius), nsample, new_xyz, xyz, idx)


def group_points_wrapper(b, c, n, npoints, nsample, points, idx, out):
    return _ops().group_points_wrapper(b, c, n, npoints, nsample, points, idx, out)


def group_points_grad_wrapper(b, c, n, npoints, nsample, grad_out, idx, grad_points):
    return _ops().group_points_grad_wrapper(b, c, n, npoints, nsample, grad_out, idx,
                                            grad_points)


def gather_points_wrapper(b, c, n, npoints, points, idx, out):
    return _ops().gather_points_wrapper(b, c, n, npoints, points, idx, out)


def gather_points_grad_wrapper(b, c, n, npoints, grad_out, idx, grad_points):
    return _ops().gather_points_grad_wrapper(b, c, n, npoints, grad_out, idx, grad_points)


def furthest_point_sampling_wrapper(b, n, m, points, temp, idx):
    return _ops().furthest_point_sampling_wrapper(b, n, m, points, temp, idx)


def three_nn_wrapper(b, n, m, unknown, known, dist2, idx):
    _ops().three_nn_wrapper(b, n, m, unknown, known, dist2, idx)


def three_interpolate_wrapper(b, c, m, n, points, idx, weight, out):
    _ops().three_interpolate_wrapper(b, c, m, n, points, idx, weight, out)


def three_interpolate_grad_wrapper(b, c, n, m, grad_out, idx, weight, grad_points):
    _ops().three_interpolate_grad_wrapper(b, c, n, m, grad_out, idx, weight, grad_points)
