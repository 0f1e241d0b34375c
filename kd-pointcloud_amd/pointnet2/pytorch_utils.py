"""Shared-MLP building blocks of the reference's pointnet2/pytorch_utils.py.

Same classes, constructor signatures, module trees and state_dict keys as the reference
(pytorch_utils.py:5-240: `SharedMLP` -> `layer{i}` -> `conv` / `bn.bn` / `activation`), so
checkpoints of the reference's PointNet++ modules load unchanged.  The channel-major
`forward` (nn.Sequential over (B, C, S, K)) is kept for API compatibility; the modules in
pointnet2_modules.py instead call `SharedMLP.cl()`, which evaluates the same layers on a
point-major (..., C) tensor: every 1x1 conv is one GEMM over all rows (dense.linear, split-K
weight gradient), and a train-mode BatchNorm followed by ReLU/LeakyReLU is one fused
statistics + normalise + activation kernel (csrc/batchnorm.hip), instead of the reference's
NCHW Conv2d / BatchNorm2d / ReLU chain.
"""
from typing import List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from dense import linear


class SharedMLP(nn.Sequential):
    """Reference: pytorch_utils.py:5-32."""

    def __init__(self, args: List[int], *, bn: bool = False, activation=nn.ReLU(inplace=True),
                 preact: bool = False, first: bool = False, name: str = "",
                 instance_norm: bool = False):
        super().__init__()
        for i in range(len(args) - 1):
            plain = not first or not preact or (i != 0)
            self.add_module(name + "layer{}".format(i),
                            Conv2d(args[i], args[i + 1], bn=plain and bn,
                                   activation=activation if plain else None, preact=preact,
                                   instance_norm=instance_norm))

    def cl(self, x):
        """The MLP on a point-major tensor (..., C_in) -> (..., C_out)."""
        for layer in self:
            x = layer.cl(x)
        return x


class _ConvBase(nn.Sequential):
    """Reference: pytorch_utils.py:35-101 (conv -> bn -> activation -> instance norm, or the
    pre-activation order)."""

    def __init__(self, in_size, out_size, kernel_size, stride, padding, activation, bn, init,
                 conv=None, batch_norm=None, bias=True, preact=False, name="",
                 instance_norm=False, instance_norm_func=None):
        super().__init__()
        bias = bias and (not bn)
        conv_unit = conv(in_size, out_size, kernel_size=kernel_size, stride=stride,
                         padding=padding, bias=bias)
        init(conv_unit.weight)
        if bias:
            nn.init.constant_(conv_unit.bias, 0)
        size = in_size if preact else out_size
        bn_unit = batch_norm(size) if bn else None
        in_unit = (instance_norm_func(size, affine=False, track_running_stats=False)
                   if instance_norm else None)
        if preact:
            if bn:
                self.add_module(name + "bn", bn_unit)
            if activation is not None:
                self.add_module(name + "activation", activation)
            if not bn and instance_norm:
                self.add_module(name + "in", in_unit)
        self.add_module(name + "conv", conv_unit)
        if not preact:
            if bn:
                self.add_module(name + "bn", bn_unit)
            if activation is not None:
                self.add_module(name + "activation", activation)
            if not bn and instance_norm:
                self.add_module(name + "in", in_unit)
        self._preact = preact

    def _pointwise(self):
        conv = next(m for m in self if isinstance(m, (nn.Conv1d, nn.Conv2d)))
        k = conv.kernel_size
        return (all(v == 1 for v in k) and all(v == 1 for v in conv.stride)
                and all(v == 0 for v in conv.padding) and conv.groups == 1)

    def cl(self, x):
        """Point-major evaluation of this unit on (..., C_in) (the reference's NCHW/NCL
        semantics: BN statistics per channel over all other dims, instance norm per batch
        element and channel over the spatial dims)."""
        if not self._pointwise():
            return _channel_major(self, x)
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, (nn.Conv1d, nn.Conv2d)):
                w = m.weight.view(m.out_channels, m.in_channels)
                x = linear(x, w, m.bias)
            elif isinstance(m, _BNBase):
                slope = _slope(nxt)
                if slope is not None and _fused_bn_ok(m[0], x):
                    x = _bn_act(m[0], slope, x)
                    i += 1  # activation consumed
                else:
                    x = _bn_rows(m[0], x)
            elif isinstance(m, (nn.InstanceNorm1d, nn.InstanceNorm2d)):
                x = _instance_norm_cl(m, x)
            else:
                x = _act(m, x)
            i += 1
        return x


def _channel_major(unit, x):
    """Fallback for non-1x1 convs: move channels to dim 1 and run the nn.Sequential."""
    d = x.dim()
    y = unit(x.movedim(-1, 1))
    return y.movedim(1, -1) if d == y.dim() else y


def _slope(act):
    if isinstance(act, nn.ReLU):
        return 0.0
    if isinstance(act, nn.LeakyReLU):
        return float(act.negative_slope)
    return None


def _fused_bn_ok(bn, x):
    from pointconv_util import _FUSED_BN
    return (_FUSED_BN and x.is_cuda and x.dtype == torch.float32 and bn.affine
            and bn.training and bn.track_running_stats and bn.momentum is not None
            and x.shape[-1] % 4 == 0 and x.shape[-1] <= 1024)


def _bn_act(bn, slope, x):
    from pointconv_util import _bn_lrelu
    return _bn_lrelu(bn, slope, x)


def _bn_rows(bn, x):
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if x2.shape[0] == 0:
        return x
    # BatchNorm{1,2}d on (R, C) rows: the per-channel statistics of the NC... layout
    y = F.batch_norm(x2, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                     bn.training or not bn.track_running_stats,
                     0.0 if bn.momentum is None else bn.momentum, bn.eps)
    if bn.training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    return y.view(shp)


def _instance_norm_cl(m, x):
    """InstanceNorm (affine=False, no running stats) of a point-major (B, ..., C) tensor:
    per (b, c) over all middle dims, biased variance."""
    b, c = x.shape[0], x.shape[-1]
    x3 = x.reshape(b, -1, c)
    mean = x3.mean(1, keepdim=True)
    var = x3.var(1, unbiased=False, keepdim=True)
    return ((x3 - mean) / torch.sqrt(var + m.eps)).view(x.shape)


def _act(m, x):
    if isinstance(m, nn.ReLU):
        return F.relu(x)
    if isinstance(m, nn.LeakyReLU):
        return F.leaky_relu(x, m.negative_slope)
    return m(x)


class _BNBase(nn.Sequential):
    """Reference: pytorch_utils.py:104-111 (weight 1, bias 0)."""

    def __init__(self, in_size, batch_norm=None, name=""):
        super().__init__()
        self.add_module(name + "bn", batch_norm(in_size))
        nn.init.constant_(self[0].weight, 1.0)
        nn.init.constant_(self[0].bias, 0)


class BatchNorm1d(_BNBase):
    def __init__(self, in_size: int, *, name: str = ""):
        super().__init__(in_size, batch_norm=nn.BatchNorm1d, name=name)


class BatchNorm2d(_BNBase):
    def __init__(self, in_size: int, name: str = ""):
        super().__init__(in_size, batch_norm=nn.BatchNorm2d, name=name)


class Conv1d(_ConvBase):
    """Reference: pytorch_utils.py:126-160."""

    def __init__(self, in_size: int, out_size: int, *, kernel_size: int = 1, stride: int = 1,
                 padding: int = 0, activation=nn.ReLU(inplace=True), bn: bool = False,
                 init=nn.init.kaiming_normal_, bias: bool = True, preact: bool = False,
                 name: str = "", instance_norm=False):
        super().__init__(in_size, out_size, kernel_size, stride, padding, activation, bn, init,
                         conv=nn.Conv1d, batch_norm=BatchNorm1d, bias=bias, preact=preact,
                         name=name, instance_norm=instance_norm,
                         instance_norm_func=nn.InstanceNorm1d)


class Conv2d(_ConvBase):
    """Reference: pytorch_utils.py:163-197."""

    def __init__(self, in_size: int, out_size: int, *, kernel_size: Tuple[int, int] = (1, 1),
                 stride: Tuple[int, int] = (1, 1), padding: Tuple[int, int] = (0, 0),
                 activation=nn.ReLU(inplace=True), bn: bool = False,
                 init=nn.init.kaiming_normal_, bias: bool = True, preact: bool = False,
                 name: str = "", instance_norm=False):
        super().__init__(in_size, out_size, kernel_size, stride, padding, activation, bn, init,
                         conv=nn.Conv2d, batch_norm=BatchNorm2d, bias=bias, preact=preact,
                         name=name, instance_norm=instance_norm,
                         instance_norm_func=nn.InstanceNorm2d)


class FC(nn.Sequential):
    """Reference: pytorch_utils.py:200-240."""

    def __init__(self, in_size: int, out_size: int, *, activation=nn.ReLU(inplace=True),
                 bn: bool = False, init=None, preact: bool = False, name: str = ""):
        super().__init__()
        fc = nn.Linear(in_size, out_size, bias=not bn)
        if init is not None:
            init(fc.weight)
        if not bn:
            nn.init.constant_(fc.bias, 0)
        if preact:
            if bn:
                self.add_module(name + "bn", BatchNorm1d(in_size))
            if activation is not None:
                self.add_module(name + "activation", activation)
        self.add_module(name + "fc", fc)
        if not preact:
            if bn:
                self.add_module(name + "bn", BatchNorm1d(out_size))
            if activation is not None:
                self.add_module(name + "activation", activation)
