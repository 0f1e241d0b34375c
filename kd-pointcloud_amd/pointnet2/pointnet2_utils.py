"""Drop-in for the reference's pointnet2/pointnet2_utils.py on gfx950 HIP kernels.

Same public names, argument meaning, shapes, dtypes and differentiability as the reference
(pointnet2_utils.py:10-290); the native calls go through the C ABI (include/kdpc.h) via
kdpc_native instead of the pybind module `pointnet2_cuda`.  Differences, all deliberate:
  * backward passes are deterministic gather-sums over an inverted index (the reference
    accumulated with float atomicAdd, pointnet2_utils.py:67-69,146-149,190-193);
  * inputs are validated (device / dtype / contiguity) with exceptions, not asserts;
  * there is no CPU path: CPU tensors raise.
"""
from typing import Tuple

import torch
import torch.nn as nn
from torch.autograd import Function

import kdpc_native as _nat


class FurthestPointSampling(Function):
    """Reference: pointnet2_utils.py:10-33 (temp filled with 1e10, int32 output)."""

    @staticmethod
    def forward(ctx, xyz: torch.Tensor, npoint: int) -> torch.Tensor:
        """xyz (B,N,3) -> (B,npoint) int32 indices of iterative furthest points."""
        return _nat.furthest_point_sampling(xyz, npoint)

    @staticmethod
    def backward(ctx, a=None):
        return None, None


furthest_point_sample = FurthestPointSampling.apply


class GatherOperation(Function):
    """Reference: pointnet2_utils.py:39-70."""

    @staticmethod
    def forward(ctx, features: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        """features (B,C,N), idx (B,npoint) int32 -> (B,C,npoint)."""
        out = _nat.gather_points(features, idx)
        ctx.save_for_backward(idx)
        ctx.n = features.shape[2]
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (idx,) = ctx.saved_tensors
        B, C, _ = grad_out.shape
        csr = _nat.csr_of(idx, ctx.n)
        return _nat.csr_sum_channels(grad_out, csr, B, C, ctx.n), None


gather_operation = GatherOperation.apply


class ThreeNN(Function):
    """Reference: pointnet2_utils.py:76-102 (returns the sqrt of the squared distances)."""

    @staticmethod
    def forward(ctx, unknown: torch.Tensor, known: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        dist2, idx = _nat.three_nn(unknown, known)
        return torch.sqrt(dist2), idx

    @staticmethod
    def backward(ctx, a=None, b=None):
        return None, None


three_nn = ThreeNN.apply


class ThreeInterpolate(Function):
    """Reference: pointnet2_utils.py:108-150."""

    @staticmethod
    def forward(ctx, features: torch.Tensor, idx: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
        """features (B,C,M), idx/weight (B,N,3) -> (B,C,N)."""
        ctx.save_for_backward(idx, weight)
        ctx.m = features.shape[2]
        return _nat.three_interpolate(features, idx, weight)

    @staticmethod
    def backward(ctx, grad_out):
        idx, weight = ctx.saved_tensors
        return _nat.three_interpolate_grad(grad_out, idx, weight, ctx.m), None, None


three_interpolate = ThreeInterpolate.apply


class GroupingOperation(Function):
    """Reference: pointnet2_utils.py:156-194."""

    @staticmethod
    def forward(ctx, features: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        """features (B,C,N), idx (B,npoint,nsample) int32 -> (B,C,npoint,nsample)."""
        ctx.save_for_backward(idx)
        ctx.n = features.shape[2]
        return _nat.group_points(features, idx)

    @staticmethod
    def backward(ctx, grad_out):
        (idx,) = ctx.saved_tensors
        B, C = grad_out.shape[:2]
        csr = _nat.csr_of(idx, ctx.n)
        return _nat.csr_sum_channels(grad_out, csr, B, C, ctx.n), None


grouping_operation = GroupingOperation.apply


class BallQuery(Function):
    """Reference: pointnet2_utils.py:200-225."""

    @staticmethod
    def forward(ctx, radius: float, nsample: int, xyz: torch.Tensor, new_xyz: torch.Tensor) -> torch.Tensor:
        """-> (B,npoint,nsample) int32: first nsample points (by index) inside the ball."""
        return _nat.ball_query(radius, nsample, xyz, new_xyz)

    @staticmethod
    def backward(ctx, a=None):
        return None, None, None, None


ball_query = BallQuery.apply


class QueryAndGroup(nn.Module):
    """Reference: pointnet2_utils.py:231-264."""

    def __init__(self, radius: float, nsample: int, use_xyz: bool = True):
        super().__init__()
        self.radius, self.nsample, self.use_xyz = radius, nsample, use_xyz

    def forward(self, xyz: torch.Tensor, new_xyz: torch.Tensor, features: torch.Tensor = None):
        idx = ball_query(self.radius, self.nsample, xyz, new_xyz)
        grouped_xyz = grouping_operation(xyz.transpose(1, 2).contiguous(), idx)
        grouped_xyz = grouped_xyz - new_xyz.transpose(1, 2).unsqueeze(-1)
        if features is None:
            assert self.use_xyz, "Cannot have not features and not use xyz as a feature!"
            return grouped_xyz
        grouped_features = grouping_operation(features, idx)
        if not self.use_xyz:
            return grouped_features
        return torch.cat([grouped_xyz, grouped_features], dim=1)


class GroupAll(nn.Module):
    """Reference: pointnet2_utils.py:267-290 (pure view/cat, no kernel)."""

    def __init__(self, use_xyz: bool = True):
        super().__init__()
        self.use_xyz = use_xyz

    def forward(self, xyz: torch.Tensor, new_xyz: torch.Tensor, features: torch.Tensor = None):
        grouped_xyz = xyz.transpose(1, 2).unsqueeze(2)
        if features is None:
            return grouped_xyz
        grouped_features = features.unsqueeze(2)
        if not self.use_xyz:
            return grouped_features
        return torch.cat([grouped_xyz, grouped_features], dim=1)
