"""GPU parity of the drop-in layers, models, losses and KD step against fixtures produced by
the REFERENCE Python (tests/golden, oracle/make_fixtures.py, oracle/make_f64_fixture.py) on
identical inputs and weights.

Tolerances (north star: 1e-5 relative for fp32 features/flows and EPE3D): integer outputs
(FPS indices) exact; flows/features rtol 1e-5 with an atol of 1e-5 x the tensor's scale
(GEMM accumulation order differs between rocBLAS and the CPU reference); losses/EPE3D
rtol 1e-5.  Gradients are compared with the reference run in FLOAT64 on the same
(replayed) neighbours: per parameter, the sum and two fixed random projections within
1e-5 of the matching absolute sum (N=2048, measured round 2: <= 4.2e-7, while the fp32
reference itself is off by up to 6.3e-5), or within twice the fp32 reference's own error
where that is larger: at N=8192 the cost volume's max over K meets exact-arithmetic
near-ties (the float64 run routes a channel's gradient to the other neighbour), and the
fp32 reference deviates from float64 by up to 1.1e-4 on the cross0 chain; the biases that
feed a train-mode BatchNorm have an exactly-zero true gradient and are compared in
absolute terms.

Free-running (the build's own kNN) the only admissible difference is a near-tie neighbour
flip: the reference ranks neighbours by |q|^2+|r|^2-2q.r in fp32, whose rounding (~1e-4 at
|q|^2 ~ 1e3) exceeds the gap between near-tied neighbours, so a last-bit difference in an
upstream warped coordinate re-ranks a few of them (and the reference's CPU GEMM rounds the
3-term dot products its own way, so exact inputs can rank a tie differently too).
test_model_free_running_* checks, at the metric's N=8192, that every neighbour-set
difference is such a tie (or a moved input downstream of one), that EPE3D and the losses
stay within 1e-5, and that pointwise flow deviations stay within the decoder's influence
radius of the flipped rows."""
import os

import numpy as np
import pytest
import torch

from weights import load_synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _close(got, want, rtol=1e-5, name=""):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    scale = max(float(np.abs(want).max()), 1e-6)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * scale, err_msg=name)


def test_layers_match_reference(golden):
    import pointconv_util as P
    g = golden("layers_ref.npz")
    x1 = _t(g["x1"].transpose(0, 2, 1)).permute(0, 2, 1)
    x2 = _t(g["x2"].transpose(0, 2, 1)).permute(0, 2, 1)
    layer = load_synthetic(P.PointConvD(256, 16, 32 + 3, 64), seed=31).to(DEV)
    nx, nf, fidx = layer(x1, _t(g["pcd_feat"]))
    np.testing.assert_array_equal(fidx.cpu().numpy(), g["pcd_fps"])
    np.testing.assert_array_equal(nx.cpu().numpy(), g["pcd_new_xyz"])
    _close(nf, g["pcd_out"], name="PointConvD")
    layer = load_synthetic(P.CrossLayerLight(32, 64, [32, 32], [32, 32]), seed=32).to(DEV)
    a, b, c = layer(x1, x2, _t(g["cl_f1"]), _t(g["cl_f2"]))
    _close(a, g["cl_out1"], name="cross f1")
    _close(b, g["cl_out2"], name="cross f2")
    _close(c, g["cl_out3"], name="cross final")
    sparse = _t(np.ascontiguousarray(g["x1"][:, :, :256].transpose(0, 2, 1))).permute(0, 2, 1)
    _close(P.UpsampleFlow()(x1, sparse, _t(g["up_sparse_flow"])), g["up_out"], name="upsample")
    _close(P.PointWarping()(x1, x2, _t(g["warp_flow"])), g["warp_out"], name="warping")
    est = load_synthetic(P.SceneFlowEstimatorResidual(32 + 32, 32), seed=33).to(DEV).train()
    fo, flo = est(x1, _t(g["est_feats"]), _t(g["est_cost"]), _t(g["warp_flow"]))
    _close(fo, g["est_out_feats"], rtol=2e-5, name="estimator feats")
    _close(flo, g["est_out_flow"], rtol=2e-5, name="estimator flow")


@pytest.mark.parametrize("name", ["fe32", "fe64", "fe128", "fe256", "pcf"])
def test_flow_layers_match_reference(golden, name):
    """FlowEmbeddingLayer (D 32 / 64: cost_volume.hip; 128 / 256: the fused wide kernels of
    cost_volume_wide.hip, D = 256 being the models' level-3 width) and
    PointConvFlow vs the reference at B=2, N=512: the output at 1e-5 of its scale, every input
    and parameter gradient of sum(out * weight) at 1e-4 of its scale (the reference's CPU GEMMs
    and the max-over-K routing accumulate in other orders)."""
    import pointconv_util as P
    from gradproj import flow_layer_weight
    g = golden("flow_layers_ref.npz")
    make = {"fe32": lambda: P.FlowEmbeddingLayer(32, 64, [32, 32]),
            "fe64": lambda: P.FlowEmbeddingLayer(32, 64, [64, 64]),
            "fe128": lambda: P.FlowEmbeddingLayer(16, 64, [128, 128]),
            "fe256": lambda: P.FlowEmbeddingLayer(16, 64, [256, 256]),
            "pcf": lambda: P.PointConvFlow(16, 64 + 64 + 3, [64, 64])}[name]
    seed = {"fe32": 51, "fe64": 52, "fe128": 53, "fe256": 55, "pcf": 54}[name]
    layer = load_synthetic(make(), seed=seed).to(DEV)
    x1 = _t(g["x1"].transpose(0, 2, 1)).permute(0, 2, 1)
    x2 = _t(g["x2"].transpose(0, 2, 1)).permute(0, 2, 1)
    ins = [t.detach().clone().requires_grad_(True) for t in (x1, x2, _t(g["f1"]), _t(g["f2"]))]
    # the reference's neighbours, replayed in call order; the build's own kNN may differ from
    # them only on near-tied rows (checked: every differing row is a near-tie of the
    # reference's fp32 distances)
    ref_idx = [g[f"{name}_knn{i}"].astype(np.int32) for i in range(2) if f"{name}_knn{i}" in g]
    calls = []

    def replay(nsample, xyz, new_xyz):
        i = len(calls)
        calls.append(1)
        own = P._nat.knn_point(nsample, xyz.contiguous(), new_xyz.contiguous()).cpu().numpy()
        ref = ref_idx[i]
        assert ref.shape == own.shape, (ref.shape, own.shape)
        xr = xyz.detach().double().cpu().numpy()
        xq = new_xyz.detach().double().cpu().numpy()
        for b, s_ in zip(*np.nonzero((np.sort(own, -1) != np.sort(ref, -1)).any(-1))):
            q = xq[b, s_]
            d = ((xr[b] - q) ** 2).sum(-1)
            lost = np.setdiff1d(ref[b, s_], own[b, s_])
            got = np.setdiff1d(own[b, s_], ref[b, s_])
            gap = abs(d[lost].max() - d[got].min())
            assert gap <= _tie_tol(q, xr[b]), (name, i, b, s_, gap)
        return _t(ref)
    prev = P.set_knn_override(replay)
    try:
        out = layer(*ins)
    finally:
        P.set_knn_override(prev)
    assert len(calls) == len(ref_idx)
    _close(out, g[name + "_out"], name=name + " out")
    (out * _t(flow_layer_weight(name, tuple(out.shape)))).sum().backward()
    for k, t in zip(("dx1", "dx2", "df1", "df2"), ins):
        _close(t.grad, g[f"{name}_{k}"], rtol=1e-4, name=f"{name} {k}")
    for k, prm in layer.named_parameters():
        if prm.grad is not None:
            _close(prm.grad, g[f"{name}_grad_{k}"], rtol=1e-4, name=f"{name} {k}")


def test_cross_layer_fg_matches_reference(golden):
    """CrossLayerLightFG (feature-space + coordinate neighbourhoods) vs the reference at B=2,
    N=512 with the reference's neighbours replayed (the build's own feature kNN agrees with
    them except on near-ties, checked): the three outputs at 1e-5 of their scale, every input
    and parameter gradient at 1e-4."""
    import pointconv_util as P
    from gradproj import flow_layer_weight
    g = golden("fg_ref.npz")
    layer = load_synthetic(P.CrossLayerLightFG(32, 64, [32, 32], [32, 32]), seed=55).to(DEV)
    x1 = _t(g["x1"].transpose(0, 2, 1)).permute(0, 2, 1)
    x2 = _t(g["x2"].transpose(0, 2, 1)).permute(0, 2, 1)
    ins = [t.detach().clone().requires_grad_(True) for t in (x1, x2, _t(g["f1"]), _t(g["f2"]))]
    # reference calls: cross(1,2): feature knn0, coords knn1; cross(2,1): knn2, knn3; the
    # build batches both directions: feature = cat(knn0, knn2), coords = cat(knn1, knn3)
    want = [np.concatenate([g["knn0"], g["knn2"]]), np.concatenate([g["knn1"], g["knn3"]])]
    np.testing.assert_array_equal(g["knn4"], g["knn0"])  # the refinement repeats cross(1,2)'s
    np.testing.assert_array_equal(g["knn5"], g["knn1"])
    calls = []

    def replay(nsample, xyz, new_xyz):
        ref = want[len(calls)].astype(np.int32)
        calls.append(xyz.shape[-1])
        own = (P._nat.knn_feature(nsample, xyz, new_xyz) if xyz.shape[-1] != 3 else
               P._nat.knn_point(nsample, xyz.contiguous(), new_xyz.contiguous())).cpu().numpy()
        assert own.shape == ref.shape
        xr = xyz.detach().double().cpu().numpy()
        xq = new_xyz.detach().double().cpu().numpy()
        d = xr.shape[-1]
        for b, s_ in zip(*np.nonzero((np.sort(own, -1) != np.sort(ref, -1)).any(-1))):
            q = xq[b, s_]
            dd = ((xr[b] - q) ** 2).sum(-1)
            lost = dd[np.setdiff1d(ref[b, s_], own[b, s_])].max()
            got = dd[np.setdiff1d(own[b, s_], ref[b, s_])].min()
            tol = 8 * d * 2.0 ** -24 * ((q ** 2).sum() + (xr[b] ** 2).sum(-1).max())
            assert abs(lost - got) <= tol, (len(calls), b, s_, lost, got)
        return _t(ref)
    prev = P.set_knn_override(replay)
    try:
        outs = layer(*ins, _t(g["k1"]), _t(g["k2"]))
    finally:
        P.set_knn_override(prev)
    assert calls == [32, 3]
    loss = 0
    for i, o in enumerate(outs):
        _close(o, g[f"out{i}"], name=f"fg out{i}")
        loss = loss + (o * _t(flow_layer_weight(f"fg{i}", tuple(o.shape)))).sum()
    loss.backward()
    for k, t in zip(("dx1", "dx2", "df1", "df2"), ins):
        _close(t.grad, g[k], rtol=1e-4, name=f"fg {k}")
    for k, prm in layer.named_parameters():
        if prm.grad is not None:
            _close(prm.grad, g[f"grad_{k}"], rtol=1e-4, name=f"fg {k}")


def test_multiscale_loss_matches_reference(golden):
    """BASELINE configs[0]: the product multiScaleLoss (HIP row gather for the GT pyramid) on
    the reference's own B=2, N=2048 four-level pyramid."""
    import loss_functions as L
    g = golden("multiscale_loss_ref.npz")
    preds = [_t(g[f"pred{i}"]) for i in range(4)]
    fps = [_t(g[f"fps{i}"]) for i in range(3)]
    loss = L.multiScaleLoss(preds, _t(g["gt"]), fps)
    np.testing.assert_allclose(loss.cpu().numpy(), g["loss"], rtol=1e-6)


# ------------------------------------------------------------------------ kNN replay
class _KnnReplay:
    """Serve every knn_point call with the index the reference computed for the same
    (K, reference cloud, query cloud), matched by coordinate checksums per batch element."""

    def __init__(self, g=None, recs=None):
        self.recs = _trace(g) if recs is None else recs
        self.worst = 0.0

    def __call__(self, nsample, xyz, new_xyz):
        x = xyz.detach().double().cpu().numpy()
        q = new_xyz.detach().double().cpu().numpy()
        out = []
        for b in range(x.shape[0]):
            i, err = _match(self.recs, nsample, x[b], q[b])
            assert i is not None, (nsample, x.shape, q.shape)
            self.worst = max(self.worst, err)
            out.append(self.recs[i][3])
        return torch.from_numpy(np.stack(out)).to(xyz.device)


def _trace(g):
    return [(int(g[f"knn{i}_k"]), g[f"knn{i}_rsum"], g[f"knn{i}_qsum"],
             g[f"knn{i}_idx"].astype(np.int32)) for i in range(int(g["n_calls"]))]


def _checksum(p):
    return np.concatenate([p.sum(0), (p ** 2).sum(0)])


def _match(recs, k, x, q):
    """Closest recorded call with this K and shape: (index, relative checksum error)."""
    rs, qs = _checksum(x), _checksum(q)
    best, err = None, np.inf
    for i, (kk, rr, qq, idx) in enumerate(recs):
        if kk != k or idx.shape != (q.shape[0], k):
            continue
        e = np.abs(rr - rs).max() / (np.abs(rr).max() + 1) + \
            np.abs(qq - qs).max() / (np.abs(qq).max() + 1)
        if e < err:
            best, err = i, e
    return best, err


class _AmaxReplay:
    """Serve the student's cost-volume max routing from the float64 reference run (its 12
    CrossLayerLight.cross calls in order; the build runs each level's two directions as one
    batch of 2B, then the refinement)."""

    def __init__(self, g64):
        self.recs = [g64[f"amax{j}"] for j in range(int(g64["n_amax"]))]
        self.pos = 0
        self.changed = 0
        self.per_call = []

    def __call__(self, amax):
        n = amax.shape[0]  # 2 (both directions, B=1) or 1 (refinement)
        ref = np.ascontiguousarray(np.concatenate(self.recs[self.pos:self.pos + n], 0))
        self.pos += n
        assert ref.shape == tuple(amax.shape), (ref.shape, amax.shape)
        out = torch.from_numpy(ref).to(amax.device)
        ch = int((out != amax).sum())
        self.changed += ch
        self.per_call.append((tuple(amax.shape), ch))
        return out


class _CvReplay(_AmaxReplay):
    """The float64 reference run's discrete cost-volume decisions, replayed into the HIP
    kernels (pointconv_util.set_cv_decisions): its max routing (_AmaxReplay) and its
    LeakyReLU decisions at near-ties.

    At LeakyReLU's kink (pre-activation 0) the derivative jumps from 0.1 to 1: like the max
    routing, a discrete choice.  The float64 fixture lists, per cost-volume call, every
    first-activation pre-activation z0 and every maximum over K of the second activation's
    pre-activation z1 that lies within 1e-4 of the call's scale of 0, with its float64 sign
    (oracle/make_f64_fixture.py); every other pre-activation is far enough from 0 that fp32
    rounding cannot move it across.  The listed z0 decisions reach the backward kernels
    through slope0 (B,N1,K,Din) u8 (1: slope 1, 2: slope 0.1), the listed z1 decisions through
    the tensor whose sign the backward reads the second derivative from (the output, with
    +-1 at the listed positions).  Every call runs the fused HIP kernels (no call is computed
    any other way; the BLAS-GEMM path of the other widths refuses a slope0); `calls` counts
    them, `replayed` the listed z0 / z1 decisions imposed."""

    def __init__(self, g64):
        super().__init__(g64)
        n = len(self.recs)
        self.z0 = [(g64[f"z0tie{j}_nkd"], g64[f"z0tie{j}_sign"]) for j in range(n)]
        self.z1 = [(g64[f"z1tie{j}_nd"], g64[f"z1tie{j}_sign"]) for j in range(n)]
        self.calls = 0
        self.replayed = [0, 0]  # listed z0 / z1 decisions imposed

    def __call__(self, amax, out, k, din):
        js = list(range(self.pos, self.pos + amax.shape[0]))
        am = super().__call__(amax)
        B, N1, _ = amax.shape
        s0 = torch.zeros((B, N1, k, din), dtype=torch.uint8, device=amax.device)
        out_b = out.clone()
        for b, jc in enumerate(js):
            nkd, sg = self.z0[jc]
            if len(nkd):
                n_, k_, d_ = (torch.from_numpy(c.astype(np.int64)).to(DEV) for c in nkd.T)
                s0[b, n_, k_, d_] = torch.from_numpy(np.where(sg > 0, 1, 2).astype(np.uint8)).to(DEV)
                self.replayed[0] += len(nkd)
            nd, sg1 = self.z1[jc]
            if len(nd):
                n_, d_ = (torch.from_numpy(c.astype(np.int64)).to(DEV) for c in nd.T)
                out_b[b, n_, d_] = torch.from_numpy(np.where(sg1 > 0, 1.0, -1.0)).float().to(DEV)
                self.replayed[1] += len(nd)
        self.calls += 1
        return am, out_b, s0


def _run_models(g, override=None, decisions=None):
    """Teacher (eval) + student (train) forward, multiScaleLoss, KD loss and its backward on
    the fixture's pair (B=1), with knn_point optionally routed through `override` and the
    student's cost-volume decisions through `decisions` (set_cv_decisions)."""
    import loss_functions as L
    import pointconv_util as P
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    pos1, pos2, flow = _t(g["pos1"]), _t(g["pos2"]), _t(g["flow"])
    prev = P.set_knn_override(override) if override is not None else None
    prev_d = P.set_cv_decisions(decisions)
    try:
        teacher = load_synthetic(Teacher(), seed=1).to(DEV).eval()
        student = load_synthetic(Student(), seed=2).to(DEV).train()
        with torch.no_grad():
            t_out = teacher(pos1, pos2, pos1, pos2)
        s_out = student(pos1, pos2, pos1, pos2)
        flows, f1i, f2i, _, _, feat1s, feat2s, _ = s_out
        msl = L.multiScaleLoss(flows, flow, f1i)
        kd = L.biDirection_loss_ht(flows, feat1s, feat2s, f1i, f2i, flow, t_out[0], t_out[5],
                                   t_out[6], t_out[1], t_out[2], 0.3, 0.8, layer=3)
        kd.backward()
    finally:
        if override is not None:
            P.set_knn_override(prev)
        P.set_cv_decisions(prev_d)
    epe_s = torch.norm(flows[0].permute(0, 2, 1) - flow, dim=2).mean()
    epe_t = torch.norm(t_out[0][0].permute(0, 2, 1) - flow, dim=2).mean()
    return dict(t=t_out, s=s_out, msl=msl, kd=kd, epe_s=epe_s, epe_t=epe_t, student=student)


def _grad_errors(student, g, g64, which="gpu"):
    """Per-parameter relative gradient errors vs the float64 reference: the sum and two
    fixed random projections, each relative to its absolute counterpart, for the build
    (which="gpu") or for the fp32 reference itself (which="ref32").  The biases that feed a
    train-mode BatchNorm are returned separately (absolute errors: their true value is 0)."""
    from gradproj import projection
    names = [n for n, _ in student.named_parameters()] if student is not None else \
        golden_names(len(g["grad_abs"]))
    assert names == list(golden_names(len(names)))
    rel, pre_bn = {}, {}
    params = dict(student.named_parameters()) if student is not None else {}
    for i, name in enumerate(names):
        if which == "gpu":
            p = params[name]
            if p.grad is None:  # the reference's never-used parameters
                assert g["grad_abs"][i] == 0.0, name
                continue
            got = float(p.grad.double().sum())
            prj = projection(name, p.grad)[0]
        else:
            if g["grad_abs"][i] == 0.0:
                continue
            got, prj = float(g["grad_sum"][i]), list(g["grad_proj"][i])
        want = float(g64["grad_sum_f64"][i])
        if name.endswith(".linear.bias") and "pointconv_list" in name:
            pre_bn[name] = abs(got - want)
            continue
        e = [abs(got - want) / max(g["grad_abs"][i], 1e-30)]
        for j in range(2):
            e.append(abs(prj[j] - g64["grad_proj_f64"][i][j]) /
                     max(g64["grad_absproj_f64"][i][j], 1e-30))
        rel[name] = max(e)
    return rel, pre_bn


def _check_grads_vs_f64(student, g, g64, tol=1e-5):
    """Every parameter's gradient error vs float64 (sum and projections) within tol; the
    pre-BatchNorm biases (true gradient 0) within 1e-5 absolute.  -> the worst error."""
    rel, pre_bn = _grad_errors(student, g, g64)
    bad = sorted(((e, n) for n, e in rel.items() if e > tol), reverse=True)
    bad += [(e, n) for n, e in pre_bn.items() if e > 1e-5]
    assert not bad, (tol, bad[:20])
    return max(rel.values())


def golden_names(n):
    """Parameter names of the fixture's student (model_ref_n4096 holds them; the trace
    fixtures follow the same module tree)."""
    import os
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "model_ref_n4096.npz"))
    names = list(ref["grad_names"])
    assert len(names) == n
    return names


@pytest.mark.parametrize("n", [2048, 8192])
def test_model_matches_reference_with_reference_neighbours(golden, n):
    """Arithmetic parity of the whole teacher/student forward, both losses, EPE3D and every
    student gradient when both sides use the same neighbour indices (the reference's,
    replayed).  n = 8192 is the metric's point count (BASELINE configs[2], B=1 here).

    Gradients are compared with the float64 reference with the float64 run's cost-volume
    max routing replayed too: where two neighbours tie within fp32 rounding the max may come
    from either, and the gradient of that (point, channel) goes to the one it came from -- a
    discrete choice, not an accumulation error (round 2, N=8192: 7 of 2.4M choices differ,
    one of them in cross3, which alone moved the level-4 gradients by 7e-4).  Without the
    routing replay the build's worst error is printed next to the fp32 reference's own."""
    g = golden(f"model_knntrace_n{n}.npz")
    g64 = golden(f"model_knntrace_n{n}_f64.npz")
    replay = _KnnReplay(g)
    r = _run_models(g, replay)
    assert replay.worst < 1e-5, replay.worst  # every call matched a recorded one
    for tag in ("t", "s"):
        out = r[tag]
        for i in range(3):
            np.testing.assert_array_equal(out[1][i].cpu().numpy(), g[f"{tag}_fps1_{i}"])
            np.testing.assert_array_equal(out[2][i].cpu().numpy(), g[f"{tag}_fps2_{i}"])
        for i in range(4):
            _close(out[0][i], g[f"{tag}_flow{i}"], name=f"{tag} flow{i}")
        _close(out[5][3], g[f"{tag}_feat1_3"], name=f"{tag} feat1s[3]")
    _close(r["msl"], g["msl"], name="multiScaleLoss")
    _close(r["kd"], g["kd"], name="KD loss")
    _close(r["epe_s"], g["s_epe3d"], name="student EPE3D")
    _close(r["epe_t"], g["t_epe3d"], name="teacher EPE3D")
    own, _ = _grad_errors(r["student"], g, g64)
    ref32, _ = _grad_errors(None, g, g64, which="ref32")
    routing = _CvReplay(g64)
    r2 = _run_models(g, _KnnReplay(g), routing)
    assert routing.pos == len(routing.recs)  # every max of the student was replayed
    assert routing.calls == 8, routing.calls  # 4 levels x (both directions + refinement)
    # 1e-5 per parameter at both sizes (the north star's fp32 bound; measured round 5: 2.2e-6
    # at N=2048, 1.5e-6 at N=8192), although at N=8192 the fp32 reference itself is up to
    # 1.6e-4 off float64 (the level-0 cost-volume chain's gradient sums cancel heavily): with
    # every discrete decision replayed, only accumulation error is left, and a regression of
    # the kernels' arithmetic shows here
    tol = 1e-5
    worst = _check_grads_vs_f64(r2["student"], g, g64, tol)
    print(f"N={n}: gradient error vs float64, HIP cost-volume kernels on all {routing.calls} "
          f"calls with the float64 max routing and LeakyReLU near-tie decisions replayed "
          f"({routing.replayed[0]} z0 / {routing.replayed[1]} z1) {worst:.2e} (bound {tol:.2e}); "
          f"with the build's own routing ({routing.changed} max choices differ: "
          f"{routing.per_call}) {max(own.values()):.2e}; fp32 reference "
          f"{max(ref32.values()):.2e}")


# --------------------------------------------------------------- free-running parity
class _KnnRecorder:
    """The build's own knn_point, recording every call (inputs and result) in order."""

    def __init__(self):
        self.calls = []

    def __call__(self, nsample, xyz, new_xyz):
        import kdpc_native
        idx = kdpc_native.knn_point(nsample, xyz.contiguous(), new_xyz.contiguous())
        self.calls.append((nsample, xyz.detach().double().cpu().numpy(),
                           new_xyz.detach().double().cpu().numpy(), idx.cpu().numpy()))
        return idx


def _tie_tol(q, r):
    """Rounding bound of the reference's expanded-form squared distance for query q against
    refs r: a few ulp of |q|^2 + |r|^2 (each of its three terms is rounded to fp32, and the
    reference's CPU GEMM may order the 3-term dot product differently), twice over."""
    return 32 * 2.0 ** -24 * ((q ** 2).sum() + (r ** 2).sum(-1).max())


def _flip_accounting(rec, g):
    """Match every kNN call of the free-running build (in program order) with the reference
    call of the same K, shape and coordinates, and explain every row whose neighbour SET
    differs, with the reference's own coordinates for that call (stored in the fixture):
      tie   -- the swapped neighbours are a near-tie of the reference's fp32 distances
               (exact inputs included: its CPU GEMM rounds the 3-term dot products its own
               way, so identical coordinates can still rank a tie differently), or
      moved -- the query or a swapped neighbour sits at a coordinate that differs from the
               reference's (a warped cloud downstream of an earlier flip).
    Returns (flip records, unexplained rows, flipped query coordinates)."""
    recs = _trace(g)
    flips, unexplained, where = [], [], []
    for ci, (k, x, q, idx) in enumerate(rec.calls):
        for b in range(x.shape[0]):
            ri, err = _match(recs, k, x[b], q[b])
            if ri is None or err > 1e-3:
                unexplained.append((ci, b, "no matching reference call", err))
                continue
            xr = g["cloud%d" % int(g[f"knn{ri}_rcloud"])].astype(np.float64)
            qr = g["cloud%d" % int(g[f"knn{ri}_qcloud"])].astype(np.float64)
            scale = np.abs(xr).max() + np.abs(qr).max()
            ours, theirs = np.sort(idx[b], -1), np.sort(recs[ri][3], -1)
            n_tie = n_moved = 0
            for row in np.nonzero((ours != theirs).any(-1))[0]:
                a = np.setdiff1d(ours[row], theirs[row])
                c = np.setdiff1d(theirs[row], ours[row])
                sw = np.concatenate([a, c])
                d = lambda s: ((xr[s] - qr[row]) ** 2).sum(-1)  # noqa: E731
                tol = _tie_tol(qr[row], xr[sw])
                moved = (np.abs(q[b][row] - qr[row]).max() > 1e-6 * scale or
                         np.abs(x[b][sw] - xr[sw]).max() > 1e-6 * scale)
                if abs(d(a).max() - d(c).min()) <= tol and abs(d(c).max() - d(a).min()) <= tol:
                    n_tie += 1
                elif moved:
                    n_moved += 1
                else:
                    unexplained.append((ci, b, int(row), d(a).tolist(), d(c).tolist(), tol))
                where.append(q[b][row])
            flips.append((ci, b, k, q.shape[1], n_tie, n_moved))
    return flips, unexplained, np.array(where).reshape(-1, 3)


@pytest.fixture(scope="module")
def free_run(golden):
    g = golden("model_knntrace_n8192.npz")
    rec = _KnnRecorder()
    r = _run_models(g, rec)
    flips, unexplained, where = _flip_accounting(rec, g)
    dump = os.environ.get("KDPC_DUMP_FREE_RUN")
    if dump:  # everything the accounting saw, for offline analysis
        d = {}
        for ci, (k, x, q, idx) in enumerate(rec.calls):
            d[f"c{ci}_k"] = np.array(k)
            d[f"c{ci}_x"], d[f"c{ci}_q"] = x.astype(np.float32), q.astype(np.float32)
            d[f"c{ci}_idx"] = idx.astype(np.int32)
        d["n_calls"] = np.array(len(rec.calls))
        for tag in ("t", "s"):
            for lv in range(4):
                d[f"{tag}_flow{lv}"] = r[tag][0][lv].detach().cpu().numpy()
        np.savez_compressed(dump, **d)
    return g, r, rec, flips, unexplained, where


def test_model_free_running_flips_are_near_ties(free_run):
    """Free-running at the metric's point count (N=8192): FPS is bit-exact, and every row
    where the build's kNN set differs from the reference trace is explained as a near-tie
    of the reference's own distances or as a moved input (see _flip_accounting)."""
    g, r, rec, flips, unexplained, where = free_run
    assert not unexplained, unexplained[:10]
    for tag in ("t", "s"):
        for i in range(3):
            np.testing.assert_array_equal(r[tag][1][i].cpu().numpy(), g[f"{tag}_fps1_{i}"])
            np.testing.assert_array_equal(r[tag][2][i].cpu().numpy(), g[f"{tag}_fps2_{i}"])
    ties = sum(f[4] for f in flips)
    moved = sum(f[5] for f in flips)
    rows = sum(rec.calls[f[0]][3].shape[1] for f in flips)
    print(f"kNN rows differing from the reference: {ties} near-ties + {moved} moved inputs "
          f"of {rows} rows in {len(flips)} (call, cloud) pairs")
    assert ties + moved < 1e-3 * rows


def _influence_radius(rec, n0):
    """How far a change at one level-0 point can travel through the level-0 decoder: the
    cost volume's K=32 neighbourhood twice (first pass + refinement) and the estimator's
    K=9 neighbourhood twice (two PointConvs), from the build's own level-0 calls."""
    r = {}
    for k, x, q, idx in rec.calls:
        if q.shape[1] == n0 and k in (9, 32):
            d = np.sqrt(((x[0][idx[0]] - q[0][:, None, :]) ** 2).sum(-1)).max()
            r[k] = max(r.get(k, 0.0), d)
    return 2 * r[32] + 2 * r[9]


def test_model_free_running_deviation_confined(free_run):
    """Free-running outputs vs the reference at N=8192.  The aggregates -- EPE3D of both
    models, multiScaleLoss, the KD loss -- within 1e-5.  Pointwise, the flows differ only
    near the flipped rows: for the eval-mode teacher every point off by more than 1e-5 of the
    flow scale lies within the decoder's influence radius of a flip; the student's train-mode
    BatchNorm couples every point through the batch statistics (a flip shifts them for all),
    so there the radius bounds the points off by more than 1e-4."""
    g, r, rec, flips, unexplained, where = free_run
    for key, want in (("msl", g["msl"]), ("kd", g["kd"]), ("epe_s", g["s_epe3d"]),
                      ("epe_t", g["t_epe3d"])):
        np.testing.assert_allclose(float(r[key]), float(want), rtol=1e-5, err_msg=key)
    n0 = g["pos1"].shape[1]
    rho = _influence_radius(rec, n0)
    report = []
    for tag, rel in (("t", 1e-5), ("s", 1e-4)):
        for lv in range(4):
            got = r[tag][0][lv][0].detach().cpu().numpy().T  # (N, 3)
            want = g[f"{tag}_flow{lv}"][0].T
            pts = r[tag][3][lv][0].detach().double().cpu().numpy().T
            scale = np.abs(want).max()
            dev = np.abs(got - want).max(-1) / scale
            off = np.nonzero(dev > rel)[0]
            far = 0.0
            if len(off):
                assert len(where), (tag, lv, "deviation without any flip")
                dist = np.sqrt(((pts[off][:, None, :] - where[None]) ** 2).sum(-1)).min(1)
                far = float(dist.max())
            report.append((tag, lv, len(off), len(dev), round(far, 3), float(dev.max())))
            assert far <= rho, (tag, lv, far, rho, report)
    print(f"influence radius {rho:.3f}; (model, level, points off, points, farthest from a "
          f"flip, max deviation / scale):", report)


# ------------------------------------------------------------- batch of 8 at N=8192
def test_batch8_n8192_fps_and_batch_independence():
    """BASELINE configs[2] size (B=8 pairs, N=8192): the encoder's FPS chain per cloud equals
    the oracle's; the eval-mode teacher's batched output equals eight single-pair runs when
    those replay the batched run's neighbours (nothing couples batch elements in eval mode;
    the GEMM libraries pick other kernels for other row counts, so free-running single runs
    may re-rank near-tied neighbours exactly as in the free-running tests above); a
    training step on the batch is finite."""
    import loss_functions as L
    import pointconv_util as P
    import pointnet2_oracle as O
    import synthetic
    from models_bid_pointconv import PointConvBidirection as Net
    p1, p2, fl = synthetic.ft3d_batch(8, 8192, seed=77)
    a, b, f = _t(p1), _t(p2), _t(fl)
    teacher = load_synthetic(Net(), seed=1).to(DEV).eval()
    fps = teacher.precompute_fps(a, b)
    x = np.concatenate([p1, p2], 0)
    for lv, idx in enumerate(fps):
        want, _ = O.furthest_point_sample(x, idx.shape[1])
        np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"FPS level {lv + 1}")
        x = np.take_along_axis(x, want[..., None].astype(np.int64), 1)
    rec = _KnnRecorder()
    prev = P.set_knn_override(rec)
    try:
        with torch.no_grad():
            out = teacher(a, b, a, b)
    finally:
        P.set_knn_override(prev)
    recs = [(k, _checksum(xx[i]), _checksum(qq[i]), idx[i])
            for k, xx, qq, idx in rec.calls for i in range(xx.shape[0])]
    for i in range(8):
        replay = _KnnReplay(recs=recs)
        prev = P.set_knn_override(replay)
        try:
            with torch.no_grad():
                one = teacher(a[i:i + 1], b[i:i + 1], a[i:i + 1], b[i:i + 1])
        finally:
            P.set_knn_override(prev)
        assert replay.worst < 1e-5, (i, replay.worst)
        for lv in range(4):
            _close(out[0][lv][i:i + 1], one[0][lv].cpu().numpy(), name=f"pair {i} flow{lv}")
    student = load_synthetic(Net(), seed=2).to(DEV).train()
    o = student(a, b, a, b)
    loss = L.multiScaleLoss(o[0], f, o[1])
    loss.backward()
    assert torch.isfinite(loss).all()
    for n, p in student.named_parameters():
        assert p.grad is None or torch.isfinite(p.grad).all(), n


# ----------------------------------------------------------------------- the KD step
def test_kd_step_matches_reference(golden):
    """distilTrain.py:164-182 through distill.KDTrainStep (the product training step: shared
    FPS chain, teacher eval/no_grad, student train, biDirection_loss_ht, backward, Adam) on
    the N=2048 trace fixture with the reference's neighbours replayed: the loss at 1e-5 and
    the gradients the optimizer sees vs the float64 reference at 1e-5, with the float64
    run's discrete cost-volume decisions (max routing, LeakyReLU near-ties) replayed as in
    test_model_matches_reference_with_reference_neighbours."""
    import pointconv_util as P
    from distill import KDTrainStep, make_optimizer
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    g = golden("model_knntrace_n2048.npz")
    g64 = golden("model_knntrace_n2048_f64.npz")
    teacher = load_synthetic(Teacher(), seed=1).to(DEV)
    student = load_synthetic(Student(), seed=2).to(DEV)
    opt = make_optimizer(student)
    seen = {}
    step_fn = opt.step

    def recording_step(*a, **k):
        for n, p in student.named_parameters():
            seen[n] = None if p.grad is None else p.grad.detach().clone()
        return step_fn(*a, **k)
    opt.step = recording_step
    before = {n: p.detach().clone() for n, p in student.named_parameters()}
    prev = P.set_knn_override(_KnnReplay(g))
    routing = _CvReplay(g64)
    prev_d = P.set_cv_decisions(routing)
    try:
        loss = KDTrainStep(teacher, student, opt)(_t(g["pos1"]), _t(g["pos2"]), _t(g["flow"]))
    finally:
        P.set_knn_override(prev)
        P.set_cv_decisions(prev_d)
    assert routing.pos == len(routing.recs)  # every max of the student was replayed
    assert routing.calls == 8, routing.calls  # every call on the HIP kernels
    print(f"KD step: gradients vs float64 with the HIP cost volume on all {routing.calls} calls "
          f"({routing.replayed[0]} z0 / {routing.replayed[1]} z1 decisions replayed)")
    _close(loss, g["kd"], name="KD loss")

    class _View:  # the recorded gradients, shaped like the module for _check_grads_vs_f64
        def named_parameters(self):
            for n, p in student.named_parameters():
                yield n, _G(seen[n])

    _check_grads_vs_f64(_View(), g, g64)
    moved = [n for n, p in student.named_parameters()
             if seen[n] is not None and not torch.equal(p.detach(), before[n])]
    assert len(moved) == sum(1 for v in seen.values() if v is not None)  # Adam stepped


class _G:
    def __init__(self, grad):
        self.grad = grad
