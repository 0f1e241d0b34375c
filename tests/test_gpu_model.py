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
upstream warped coordinate re-ranks a few of them.  test_model_free_running_* checks that
every neighbour-set difference is such a tie and that flow deviations stay inside the
neighbourhoods those flips can reach."""
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


def _run_models(g, override=None):
    """Teacher (eval) + student (train) forward, multiScaleLoss, KD loss and its backward on
    the fixture's pair (B=1), with knn_point optionally routed through `override`."""
    import loss_functions as L
    import pointconv_util as P
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    pos1, pos2, flow = _t(g["pos1"]), _t(g["pos2"]), _t(g["flow"])
    prev = P.set_knn_override(override) if override is not None else None
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
    epe_s = torch.norm(flows[0].permute(0, 2, 1) - flow, dim=2).mean()
    epe_t = torch.norm(t_out[0][0].permute(0, 2, 1) - flow, dim=2).mean()
    return dict(t=t_out, s=s_out, msl=msl, kd=kd, epe_s=epe_s, epe_t=epe_t, student=student)


def _check_grads_vs_f64(student, g, g64, tol=1e-5):
    """Per-parameter gradient sums and projections vs the float64 reference (module doc)."""
    from gradproj import projection
    names = [n for n, _ in student.named_parameters()]
    assert names == list(golden_names(len(names)))
    bad = []
    for i, (name, p) in enumerate(student.named_parameters()):
        if p.grad is None:  # the reference's never-used parameters
            assert g["grad_abs"][i] == 0.0, name
            continue
        got = float(p.grad.double().sum())
        want = float(g64["grad_sum_f64"][i])
        if name.endswith(".linear.bias") and "pointconv_list" in name:
            # d(BN(x))/d(bias of x) sums to exactly 0 over the batch: both sides are noise
            if abs(got - want) > 1e-5:
                bad.append((name, "pre-BN bias", got, want))
            continue
        ref32 = abs(float(g["grad_sum"][i]) - want)  # the reference's own fp32 error
        if abs(got - want) > max(tol * g["grad_abs"][i], 2 * ref32) + 1e-9:
            bad.append((name, "sum", got, want, float(g["grad_abs"][i]), ref32))
        prj, scale = projection(name, p.grad)
        for j in range(2):
            w, s = g64["grad_proj_f64"][i][j], g64["grad_absproj_f64"][i][j]
            ref32 = abs(float(g["grad_proj"][i][j]) - w)
            if abs(prj[j] - w) > max(tol * s, 2 * ref32) + 1e-9:
                bad.append((name, f"proj{j}", prj[j], float(w), float(s), ref32))
    assert not bad, bad[:20]


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
    replayed).  n = 8192 is the metric's point count (BASELINE configs[2], B=1 here)."""
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
    _check_grads_vs_f64(r["student"], g, g64)


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
    refs r: a few ulp of |q|^2 + |r|^2 (each of its three terms is rounded to fp32), plus the
    same again for inputs that agree with the reference's to the last bits."""
    return 32 * 2.0 ** -24 * ((q ** 2).sum() + (r ** 2).sum(-1).max())


def _cloud_of(p, pcs1, pcs2):
    """(level, side) of a point array by its size and its nearness to the level's clouds
    (derived clouds -- warped pc2, pc1 + flow -- move by about one flow, far less than the
    distance between unrelated samples)."""
    for lv in range(len(pcs1)):
        if pcs1[lv].shape[0] == p.shape[0]:
            d1 = np.abs(p - pcs1[lv]).mean()
            d2 = np.abs(p - pcs2[lv]).mean()
            return lv, (1 if d1 <= d2 else 2)
    return None


def _flip_accounting(rec, g, pcs1, pcs2):
    """Walk the build's kNN calls in program order against the reference trace.  Returns
    (taint per (level, side), per-call flip counts, unexplained flips).  A row may differ
    from the reference only if (a) its query or a neighbour in either set is already
    tainted (its inputs legitimately moved), or (b) the swapped neighbours are a near-tie
    under the expanded form's rounding; rows of kind (b) become tainted.  Taint then spreads
    two hops along every call (query <- its neighbours), a superset of the model's data
    flow through each neighbourhood."""
    recs = _trace(g)
    taint = {}
    flips, unexplained = [], []

    def tset(key, n):
        if key not in taint:
            taint[key] = np.zeros(n, bool)
        return taint[key]

    for ci, (k, x, q, idx) in enumerate(rec.calls):
        for b in range(x.shape[0]):
            ident_q, ident_r = _cloud_of(q[b], pcs1, pcs2), _cloud_of(x[b], pcs1, pcs2)
            if ident_q is None or ident_r is None:  # level-4 encoder call: exact coordinates
                continue
            tq, tr = tset(ident_q, q.shape[1]), tset(ident_r, x.shape[1])
            ri, err = _match(recs, k, x[b], q[b])
            nflip = 0
            if ri is not None and err < 1e-3:
                ref_idx = recs[ri][3]
                ours = np.sort(idx[b], -1)
                theirs = np.sort(ref_idx, -1)
                for row in np.nonzero((ours != theirs).any(-1))[0]:
                    a = np.setdiff1d(ours[row], theirs[row])
                    c = np.setdiff1d(theirs[row], ours[row])
                    if tq[row] or tr[a].any() or tr[c].any():
                        continue  # inputs already moved by an upstream flip
                    d = lambda s: ((x[b][s] - q[b][row]) ** 2).sum(-1)  # noqa: E731
                    tol = _tie_tol(q[b][row], x[b][np.concatenate([a, c])])
                    if abs(d(a).max() - d(c).min()) > tol or abs(d(c).max() - d(a).min()) > tol:
                        unexplained.append((ci, b, int(row), d(a).tolist(), d(c).tolist(), tol))
                    tq[row] = True
                    nflip += 1
            else:
                unexplained.append((ci, b, "no matching reference call", err))
            flips.append((ci, k, ident_q, ident_r, nflip))
            for _ in range(2):  # (tq is tr for a self-kNN: two hops through the cloud)
                tq |= tr[idx[b]].any(-1)
    return taint, flips, unexplained


@pytest.fixture(scope="module")
def free_run(golden):
    g = golden("model_knntrace_n8192.npz")
    rec = _KnnRecorder()
    r = _run_models(g, rec)
    pcs1 = [p[0].permute(1, 0).detach().double().cpu().numpy() for p in r["t"][3]]
    pcs2 = [p[0].permute(1, 0).detach().double().cpu().numpy() for p in r["t"][4]]
    taint, flips, unexplained = _flip_accounting(rec, g, pcs1, pcs2)
    dump = os.environ.get("KDPC_DUMP_FREE_RUN")
    if dump:  # everything the accounting saw, for offline analysis (tools/)
        d = {"pcs1_%d" % i: p.astype(np.float32) for i, p in enumerate(pcs1)}
        d.update({"pcs2_%d" % i: p.astype(np.float32) for i, p in enumerate(pcs2)})
        for ci, (k, x, q, idx) in enumerate(rec.calls):
            d[f"c{ci}_k"] = np.array(k)
            d[f"c{ci}_x"], d[f"c{ci}_q"] = x.astype(np.float32), q.astype(np.float32)
            d[f"c{ci}_idx"] = idx.astype(np.int32)
        d["n_calls"] = np.array(len(rec.calls))
        for tag in ("t", "s"):
            for lv in range(4):
                d[f"{tag}_flow{lv}"] = r[tag][0][lv].detach().cpu().numpy()
        np.savez_compressed(dump, **d)
    return g, r, taint, flips, unexplained


def test_model_free_running_flips_are_near_ties(free_run):
    """Every neighbour-set difference between the build's kNN and the reference trace, on a
    query whose inputs still agree with the reference, is a near-tie of the reference's own
    fp32 distance formula; FPS (exact coordinates) is bit-exact."""
    g, r, taint, flips, unexplained = free_run
    assert not unexplained, unexplained[:10]
    for tag in ("t", "s"):
        for i in range(3):
            np.testing.assert_array_equal(r[tag][1][i].cpu().numpy(), g[f"{tag}_fps1_{i}"])
            np.testing.assert_array_equal(r[tag][2][i].cpu().numpy(), g[f"{tag}_fps2_{i}"])
    total = sum(f[-1] for f in flips)
    rows = sum(1 for _ in flips)
    print(f"near-tie flips: {total} rows over {rows} (call, cloud) pairs;",
          {k: int(v.sum()) for k, v in taint.items()})


def test_model_free_running_deviation_confined(free_run):
    """Free-running flows vs the reference: the coarse level (no warping upstream) and every
    point outside the flip taint at 1e-5 of scale for the eval-mode teacher.  The student's
    train-mode BatchNorm couples all points through the batch statistics, so untainted
    student points are held to 1e-4 of scale (the statistics shift by at most the tainted
    fraction times the local deviation).  Losses and EPE3D are aggregates: 1e-4 relative."""
    g, r, taint, flips, unexplained = free_run
    report = []
    for tag, rel in (("t", 1e-5), ("s", 1e-4)):
        for lv in range(4):
            got = r[tag][0][lv][0].detach().cpu().numpy().T  # (N, 3)
            want = g[f"{tag}_flow{lv}"][0].T
            scale = np.abs(want).max()
            dev = np.abs(got - want).max(-1) > 1e-5 * scale
            t = taint.get((lv, 1), np.zeros(len(dev), bool))
            outside = dev & ~t
            report.append((tag, lv, int(dev.sum()), int(t.sum()), len(dev)))
            assert not (np.abs(got - want)[~t] > rel * scale).any(), (tag, lv, report)
            assert t.mean() < 0.25, (tag, lv, "taint covers too much of the cloud", report)
            if tag == "t":
                assert not outside.any(), (tag, lv, int(outside.sum()), report)
    print("deviating / tainted / points per (model, level):", report)
    for key, want in (("msl", g["msl"]), ("kd", g["kd"]), ("epe_s", g["s_epe3d"]),
                      ("epe_t", g["t_epe3d"])):
        np.testing.assert_allclose(float(r[key]), float(want), rtol=1e-4, err_msg=key)


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
    the gradients the optimizer sees vs the float64 reference at 1e-5."""
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
    try:
        loss = KDTrainStep(teacher, student, opt)(_t(g["pos1"]), _t(g["pos2"]), _t(g["flow"]))
    finally:
        P.set_knn_override(prev)
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
