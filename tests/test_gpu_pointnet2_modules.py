"""PointNet++ set abstraction (MSG, group-all) and feature propagation (SURVEY §8f rank 4,
ref pointnet2/pointnet2_modules.py:10-156) on the HIP path vs fixtures produced by the
REFERENCE modules (oracle/make_fixtures.py `safp`: same inputs, same synthetic weights,
train-mode BatchNorm).

FPS centroids and ball_query neighbourhoods are integer work and must agree exactly (the
new_xyz output is checked bit for bit); features at 1e-5 of their scale (the GEMMs and the
BN statistics sum in other orders than the CPU reference); gradients at 1e-4 of scale (the
max over K routes to the same first maximal neighbour, but the backward's sums are
reordered); BN running statistics at 1e-5."""
import numpy as np
import pytest
import torch

from weights import load_synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _close(got, want, rtol, name):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    scale = max(float(np.abs(want).max()), 1e-6)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * scale, err_msg=name)


def _modules():
    from pointnet2 import pointnet2_modules as M
    sa = load_synthetic(M.PointnetSAModuleMSG(npoint=128, radii=[0.2, 0.4], nsamples=[16, 32],
                                              mlps=[[6, 16, 32], [6, 16, 32]], bn=True), seed=65)
    ga = load_synthetic(M.PointnetSAModule(mlp=[64, 64, 128], npoint=None, bn=True), seed=66)
    fp = load_synthetic(M.PointnetFPModule(mlp=[64 + 6, 64, 32], bn=True), seed=67)
    return [m.to(DEV).train() for m in (sa, ga, fp)]


def test_pointnet2_modules_match_reference(golden):
    from gradproj import flow_layer_weight
    g = golden("pointnet2_modules_ref.npz")
    sa, ga, fp = _modules()
    xi = _t(g["xyz"]).requires_grad_(True)
    fi = _t(g["feats"]).requires_grad_(True)
    new_xyz, f1 = sa(xi, fi)
    np.testing.assert_array_equal(new_xyz.detach().cpu().numpy(), g["new_xyz"])
    _, f2 = ga(new_xyz, f1)
    f3 = fp(xi, new_xyz, fi, f1)
    assert f1.is_contiguous() and f2.is_contiguous() and f3.is_contiguous()
    _close(f1, g["sa_out"], 1e-5, "SA MSG out")
    _close(f2, g["ga_out"], 1e-5, "SA group-all out")
    _close(f3, g["fp_out"], 1e-5, "FP out")
    loss = 0
    for k, o in (("sa", f1), ("ga", f2), ("fp", f3)):
        loss = loss + (o * _t(flow_layer_weight(k, tuple(o.shape)))).sum()
    loss.backward()
    _close(xi.grad, g["dxyz"], 1e-4, "dxyz")
    _close(fi.grad, g["dfeats"], 1e-4, "dfeats")
    for tag, m in (("sa", sa), ("ga", ga), ("fp", fp)):
        for k, prm in m.named_parameters():
            _close(prm.grad, g[f"grad_{tag}.{k}"], 1e-4, f"{tag} {k}")
        for k, buf in m.named_buffers():
            _close(buf, g[f"buf_{tag}.{k}"], 1e-5, f"{tag} {k}")


def test_sa_eval_and_empty_balls():
    """Eval-mode SA (running statistics) equals the channel-major nn.Sequential path of the
    same modules (the reference's own forward: grouping -> Conv2d/BN2d/ReLU -> max_pool2d),
    including centroids whose ball holds only themselves (r tiny: every slot = the centre)."""
    import torch.nn.functional as F
    from pointnet2 import pointnet2_modules as M
    from pointnet2 import pointnet2_utils as U
    torch.manual_seed(3)
    sa = M.PointnetSAModuleMSG(npoint=64, radii=[1e-4, 0.3], nsamples=[8, 16],
                               mlps=[[4, 16], [4, 32]], bn=True).to(DEV).eval()
    for p in sa.parameters():
        torch.nn.init.normal_(p)
    for m in sa.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.normal_()
            m.running_var.uniform_(0.5, 2.0)
    xyz = torch.rand(2, 512, 3, device=DEV)
    feats = torch.randn(2, 4, 512, device=DEV)
    with torch.no_grad():
        new_xyz, out = sa(xyz, feats)
        ref = []
        for grouper, mlp in zip(sa.groupers, sa.mlps):
            x = U.QueryAndGroup(grouper.radius, grouper.nsample)(xyz, new_xyz, feats)
            ref.append(F.max_pool2d(mlp(x), kernel_size=[1, x.size(3)]).squeeze(-1))
        ref = torch.cat(ref, 1)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
