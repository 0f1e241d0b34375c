"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by kd-pointcloud_amd/).

numpy front-end for the C restatement in pointnet2_oracle.c.  Every function takes
and returns numpy arrays with the reference's shapes/dtypes:

  furthest_point_sample(xyz (B,N,3) f32, m)            -> (idx (B,M) i32, temp (B,N) f32)
  gather_points(points (B,C,N), idx (B,M))             -> (B,C,M)      sampling_gpu.cu:8-24
  gather_points_grad(grad_out (B,C,M), idx, n)         -> (B,C,N)      sampling_gpu.cu:46-63
  ball_query(radius, nsample, xyz (B,N,3), new_xyz)    -> (B,M,K) i32  ball_query_gpu.cu:9-45
  group_points(points (B,C,N), idx (B,S,K))            -> (B,C,S,K)    group_points_gpu.cu:47-66
  group_points_grad(grad_out (B,C,S,K), idx, n)        -> (B,C,N)      group_points_gpu.cu:8-25
  three_nn(unknown (B,N,3), known (B,M,3))             -> (dist2, idx) interpolate_gpu.cu:9-52
  three_interpolate(points (B,C,M), idx, weight)       -> (B,C,N)      interpolate_gpu.cu:77-97
  three_interpolate_grad(grad_out (B,C,N), idx, w, m)  -> (B,C,M)      interpolate_gpu.cu:120-142
  square_distance(src (B,S,3), dst (B,N,3))            -> (B,S,N)      pointconv_util.py:73-94
  knn(k, xyz (B,N,3), new_xyz (B,S,3))                 -> (idx, dist)  pointconv_util.py:96-107
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libpointnet2_oracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _fp(a):
    return a.ctypes.data_as(_f)


def _ip(a):
    return a.ctypes.data_as(_i)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ci32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def opt_n_threads(n):
    return _load().oracle_opt_n_threads(int(n))


def furthest_point_sample(xyz, m):
    xyz = _c32(xyz)
    b, n, _ = xyz.shape
    temp = np.full((b, n), 1e10, dtype=np.float32)
    idx = np.zeros((b, m), dtype=np.int32)
    _load().oracle_furthest_point_sampling(b, n, int(m), _fp(xyz), _fp(temp), _ip(idx))
    return idx, temp


def gather_points(points, idx):
    points, idx = _c32(points), _ci32(idx)
    b, c, n = points.shape
    m = idx.shape[1]
    out = np.zeros((b, c, m), dtype=np.float32)
    _load().oracle_gather_points(b, c, n, m, _fp(points), _ip(idx), _fp(out))
    return out


def gather_points_grad(grad_out, idx, n):
    grad_out, idx = _c32(grad_out), _ci32(idx)
    b, c, m = grad_out.shape
    out = np.zeros((b, c, n), dtype=np.float32)
    _load().oracle_gather_points_grad(b, c, n, m, _fp(grad_out), _ip(idx), _fp(out))
    return out


def ball_query(radius, nsample, xyz, new_xyz):
    xyz, new_xyz = _c32(xyz), _c32(new_xyz)
    b, n, _ = xyz.shape
    m = new_xyz.shape[1]
    idx = np.zeros((b, m, nsample), dtype=np.int32)
    _load().oracle_ball_query(b, n, m, ctypes.c_float(radius), int(nsample), _fp(new_xyz),
                              _fp(xyz), _ip(idx))
    return idx


def group_points(points, idx):
    points, idx = _c32(points), _ci32(idx)
    b, c, n = points.shape
    _, s, k = idx.shape
    out = np.zeros((b, c, s, k), dtype=np.float32)
    _load().oracle_group_points(b, c, n, s, k, _fp(points), _ip(idx), _fp(out))
    return out


def group_points_grad(grad_out, idx, n):
    grad_out, idx = _c32(grad_out), _ci32(idx)
    b, c, s, k = grad_out.shape
    out = np.zeros((b, c, n), dtype=np.float32)
    _load().oracle_group_points_grad(b, c, n, s, k, _fp(grad_out), _ip(idx), _fp(out))
    return out


def three_nn(unknown, known):
    unknown, known = _c32(unknown), _c32(known)
    b, n, _ = unknown.shape
    m = known.shape[1]
    dist2 = np.zeros((b, n, 3), dtype=np.float32)
    idx = np.zeros((b, n, 3), dtype=np.int32)
    _load().oracle_three_nn(b, n, m, _fp(unknown), _fp(known), _fp(dist2), _ip(idx))
    return dist2, idx


def three_interpolate(points, idx, weight):
    points, idx, weight = _c32(points), _ci32(idx), _c32(weight)
    b, c, m = points.shape
    n = idx.shape[1]
    out = np.zeros((b, c, n), dtype=np.float32)
    _load().oracle_three_interpolate(b, c, m, n, _fp(points), _ip(idx), _fp(weight), _fp(out))
    return out


def three_interpolate_grad(grad_out, idx, weight, m):
    grad_out, idx, weight = _c32(grad_out), _ci32(idx), _c32(weight)
    b, c, n = grad_out.shape
    out = np.zeros((b, c, m), dtype=np.float32)
    _load().oracle_three_interpolate_grad(b, c, n, m, _fp(grad_out), _ip(idx), _fp(weight),
                                          _fp(out))
    return out


def square_distance(src, dst):
    src, dst = _c32(src), _c32(dst)
    b, s, _ = src.shape
    n = dst.shape[1]
    out = np.zeros((b, s, n), dtype=np.float32)
    _load().oracle_square_distance(b, s, n, _fp(src), _fp(dst), _fp(out))
    return out


def knn(k, xyz, new_xyz):
    xyz, new_xyz = _c32(xyz), _c32(new_xyz)
    b, n, _ = xyz.shape
    s = new_xyz.shape[1]
    idx = np.zeros((b, s, k), dtype=np.int32)
    dist = np.zeros((b, s, k), dtype=np.float32)
    _load().oracle_knn(b, n, s, int(k), _fp(xyz), _fp(new_xyz), _ip(idx), _fp(dist))
    return idx, dist
