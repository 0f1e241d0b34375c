"""PointNet++ modules: module trees / state_dict keys equal the reference's (the keys the
reference-generated fixture recorded), constructor semantics (use_xyz widens the first MLP
width in place, as the reference does) -- CPU, no kernels run."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_state_dict_keys_match_reference():
    from pointnet2 import pointnet2_modules as M
    g = np.load(os.path.join(GOLDEN, "pointnet2_modules_ref.npz"))
    mlps = [[6, 16, 32], [6, 16, 32]]
    sa = M.PointnetSAModuleMSG(npoint=128, radii=[0.2, 0.4], nsamples=[16, 32], mlps=mlps,
                               bn=True)
    assert mlps[0][0] == 9  # widened in place by use_xyz (reference behaviour)
    ga = M.PointnetSAModule(mlp=[64, 64, 128], npoint=None, bn=True)
    fp = M.PointnetFPModule(mlp=[70, 64, 32], bn=True)
    for tag, m in (("sa", sa), ("ga", ga), ("fp", fp)):
        params = {f"grad_{tag}.{k}": tuple(p.shape) for k, p in m.named_parameters()}
        bufs = {f"buf_{tag}.{k}": tuple(b.shape) for k, b in m.named_buffers()}
        want_p = {k: g[k].shape for k in g.files if k.startswith(f"grad_{tag}.")}
        want_b = {k: g[k].shape for k in g.files if k.startswith(f"buf_{tag}.")}
        assert params == want_p, tag
        assert bufs == want_b, tag


def test_conv_without_bn_has_bias():
    from pointnet2 import pytorch_utils as pt
    c = pt.Conv2d(4, 8, bn=False)
    assert c.conv.bias is not None and float(c.conv.bias.abs().sum()) == 0.0
    c = pt.Conv2d(4, 8, bn=True)
    assert c.conv.bias is None and list(dict(c.named_children())) == ["conv", "bn", "activation"]
