"""PointNet++ set-abstraction and feature-propagation modules (reference:
pointnet2/pointnet2_modules.py:10-156) on the gfx950 kernels.

Same classes, keyword-only constructors, argument meaning, output shapes and state_dict keys
(`mlps.{i}.layer{j}.conv.weight`, `...bn.bn.*`; `mlp.layer{j}...`) as the reference.  The
reference groups channel-major -- ball_query -> grouping_operation on (B,C,N) -> (B,3+C,S,K)
-> Conv2d/BN2d/ReLU chain -> F.max_pool2d over K.  Here the set abstraction runs
point-major end to end:

  * FPS (bit-exact HIP kernel) and the centroid gather as one row gather (B,S,3);
  * ball_query (HIP, the reference's first-K-by-index semantics, empty balls -> index 0);
  * neighbour rows gathered as (B,S,K,C) (kdpc_group_rows: contiguous C-float rows per
    neighbour, deterministic CSR gather-sum backward), centred xyz first as in the
    reference's `cat([grouped_xyz, grouped_features], 1)`;
  * each 1x1 Conv2d is one GEMM over the B*S*K rows, BN2d + ReLU one fused kernel
    (SharedMLP.cl), then max (or mean) over the K neighbours;
  * the features are transposed to point-major once per call, not per grouper.

Feature propagation uses the reference's own ops (three_nn -> inverse-distance weights ->
three_interpolate, HIP, bit-exact) and runs its MLP point-major on the concatenated
features.
"""
from typing import List

import torch
import torch.nn as nn

from . import pointnet2_utils
from . import pytorch_utils as pt_utils


def _rows(points, idx):
    """points (B,N,C) gathered by idx (B,...) int32 -> (B,...,C) (autograd: CSR sum)."""
    from pointconv_util import _group_rows
    return _group_rows(points, idx)


class _PointnetSAModuleBase(nn.Module):
    """Reference: pointnet2_modules.py:10-55."""

    def __init__(self):
        super().__init__()
        self.npoint = None
        self.groupers = None
        self.mlps = None
        self.pool_method = "max_pool"

    def forward(self, xyz: torch.Tensor, features: torch.Tensor = None, new_xyz=None):
        """xyz (B,N,3), features (B,C,N) or None, new_xyz (B,S,3) or None ->
        (new_xyz (B,npoint,3), new_features (B, sum_k mlps[k][-1], npoint))."""
        if new_xyz is None and self.npoint is not None:
            fps_idx = pointnet2_utils.furthest_point_sample(xyz, self.npoint)
            new_xyz = _rows(xyz.contiguous(), fps_idx)
        feats_pm = None if features is None else features.transpose(1, 2).contiguous()
        out = []
        for grouper, mlp in zip(self.groupers, self.mlps):
            x = self._group(grouper, xyz, new_xyz, features, feats_pm)  # (B,S,K,C_in)
            h = mlp.cl(x) if isinstance(mlp, pt_utils.SharedMLP) else \
                mlp(x.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
            if self.pool_method == "max_pool":
                # F.max_pool2d over K keeps the first maximal neighbour; so does max(dim)
                h = h.max(dim=2)[0]
            elif self.pool_method == "avg_pool":
                h = h.mean(dim=2)
            else:
                raise NotImplementedError
            out.append(h)
        return new_xyz, torch.cat(out, dim=-1).transpose(1, 2).contiguous()

    @staticmethod
    def _group(grouper, xyz, new_xyz, features, feats_pm):
        if isinstance(grouper, pointnet2_utils.QueryAndGroup):
            idx = pointnet2_utils.ball_query(grouper.radius, grouper.nsample, xyz, new_xyz)
            gx = _rows(xyz.contiguous(), idx) - new_xyz.unsqueeze(2)
            if feats_pm is None:
                assert grouper.use_xyz, "Cannot have not features and not use xyz as a feature!"
                return gx
            gf = _rows(feats_pm, idx)
            return torch.cat([gx, gf], dim=-1) if grouper.use_xyz else gf
        if isinstance(grouper, pointnet2_utils.GroupAll):
            if feats_pm is None:
                return xyz.unsqueeze(1)
            if not grouper.use_xyz:
                return feats_pm.unsqueeze(1)
            return torch.cat([xyz, feats_pm], dim=-1).unsqueeze(1)
        # any other grouper: its own (B,C,S,K) output, moved to point-major
        return grouper(xyz, new_xyz, features).permute(0, 2, 3, 1)


class PointnetSAModuleMSG(_PointnetSAModuleBase):
    """Pointnet set abstraction layer with multiscale grouping (reference:
    pointnet2_modules.py:58-95)."""

    def __init__(self, *, npoint: int, radii: List[float], nsamples: List[int],
                 mlps: List[List[int]], bn: bool = True, use_xyz: bool = True,
                 pool_method="max_pool", instance_norm=False):
        super().__init__()
        assert len(radii) == len(nsamples) == len(mlps)
        self.npoint = npoint
        self.groupers = nn.ModuleList()
        self.mlps = nn.ModuleList()
        for radius, nsample, spec in zip(radii, nsamples, mlps):
            self.groupers.append(
                pointnet2_utils.QueryAndGroup(radius, nsample, use_xyz=use_xyz)
                if npoint is not None else pointnet2_utils.GroupAll(use_xyz))
            if use_xyz:
                spec[0] += 3  # the reference widens the caller's list in place
            self.mlps.append(pt_utils.SharedMLP(spec, bn=bn, instance_norm=instance_norm))
        self.pool_method = pool_method


class PointnetSAModule(PointnetSAModuleMSG):
    """Pointnet set abstraction layer (reference: pointnet2_modules.py:98-118)."""

    def __init__(self, *, mlp: List[int], npoint: int = None, radius: float = None,
                 nsample: int = None, bn: bool = True, use_xyz: bool = True,
                 pool_method="max_pool", instance_norm=False):
        super().__init__(mlps=[mlp], npoint=npoint, radii=[radius], nsamples=[nsample], bn=bn,
                         use_xyz=use_xyz, pool_method=pool_method, instance_norm=instance_norm)


class PointnetFPModule(nn.Module):
    """Propagates the features of one set to another (reference:
    pointnet2_modules.py:121-156)."""

    def __init__(self, *, mlp: List[int], bn: bool = True):
        super().__init__()
        self.mlp = pt_utils.SharedMLP(mlp, bn=bn)

    def forward(self, unknown: torch.Tensor, known: torch.Tensor, unknow_feats: torch.Tensor,
                known_feats: torch.Tensor) -> torch.Tensor:
        """unknown (B,n,3), known (B,m,3) or None, unknow_feats (B,C1,n) or None,
        known_feats (B,C2,m) -> (B, mlp[-1], n)."""
        if known is not None:
            dist, idx = pointnet2_utils.three_nn(unknown, known)
            dist_recip = 1.0 / (dist + 1e-8)
            norm = torch.sum(dist_recip, dim=2, keepdim=True)
            weight = dist_recip / norm
            interpolated = pointnet2_utils.three_interpolate(known_feats, idx, weight)
        else:
            interpolated = known_feats.expand(*known_feats.size()[0:2], unknown.size(1))
        new = interpolated if unknow_feats is None else \
            torch.cat([interpolated, unknow_feats], dim=1)  # (B, C2 + C1, n)
        return self.mlp.cl(new.transpose(1, 2)).transpose(1, 2).contiguous()
