"""BASELINE configs[3] -- the KD step of distilTrain.py:156-185 (teacher fwd in eval/no_grad,
student fwd+bwd, biDirection_loss_ht, Adam) -- at its per-GPU slice of B=32 over 8 GPUs:
B=4 pairs of N=8192 points, through the product step (distill.graphed_kd_step, the step the
bench times).  Plus the graphed step's optimizer contract (eager steps and LR changes in
between) and HIP-graph replay of the step's reductions."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(b, n, seed):
    import synthetic
    return tuple(torch.from_numpy(a).to(DEV) for a in synthetic.ft3d_batch(b, n, seed=seed))


def test_graphed_kd_step_b4_n8192():
    """FPS chain per cloud equals the oracle's; loss and gradients finite; the graphed KD
    step is bit-identical to the eager KDTrainStep (losses and parameters) over replays with
    and without an in-graph FPS prefetch."""
    import pointnet2_oracle as O
    from distill import KDTrainStep, graphed_kd_step, make_optimizer
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    torch.manual_seed(1)
    teacher = Teacher().to(DEV)
    torch.manual_seed(2)
    base = Student().to(DEV)
    batches = [_batch(4, 8192, s) for s in (31, 32, 33)]
    # FPS chain (levels 1-4, both clouds) vs the C oracle, cloud by cloud
    fps = base.precompute_fps(batches[0][0], batches[0][1])
    x = torch.cat([batches[0][0], batches[0][1]], 0).cpu().numpy()
    for lv, idx in enumerate(fps):
        want, _ = O.furthest_point_sample(x, idx.shape[1])
        np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"FPS level {lv + 1}")
        x = np.take_along_axis(x, want[..., None].astype(np.int64), 1)
    eager_model, graph_model = copy.deepcopy(base), copy.deepcopy(base)
    opt_e = make_optimizer(eager_model, capturable=True)
    opt_g = make_optimizer(graph_model, capturable=True)
    eager = KDTrainStep(teacher, eager_model, opt_e)
    graphed = graphed_kd_step(teacher, graph_model, opt_g, batches[0], warmup=1)
    eager(*batches[0])  # the graphed step's constructor ran one eager warm-up step
    seq = [(batches[1], batches[2]), (batches[2], None), (batches[1], None)]
    for b, nxt in seq:
        le = eager(*b, next_batch=nxt)
        lg = graphed(*b, next_batch=nxt)
        torch.cuda.synchronize()
        assert torch.isfinite(lg).all(), float(lg)
        assert float(le) == float(lg), (float(le), float(lg))
        assert torch.isfinite(graphed.G).all()  # the packed student gradients of this replay
    for (n, pe), pg in zip(eager_model.named_parameters(), graph_model.parameters()):
        assert torch.equal(pe, pg), n
    assert all(p.grad is None for p in teacher.parameters())  # frozen teacher


def test_graphed_step_honours_eager_steps_and_lr_changes():
    """the graphed step's flat Adam shares state with the caller's optimizer.  An
    eager step on that optimizer between replays, and an LR change by plain assignment (the
    reference's per-epoch LR clip, distilTrain.py:146-149) or by a torch scheduler, must
    reach the graph: parameters and Adam step counters equal an all-eager run."""
    from distill import FlowTrainStep, graphed_flow_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    base = PointConvBidirection().to(DEV)
    b = [_batch(1, 2048, s) for s in (41, 42, 43)]
    mg, me = copy.deepcopy(base), copy.deepcopy(base)
    og, oe = make_optimizer(mg, capturable=True), make_optimizer(me, capturable=True)
    graphed = graphed_flow_step(mg, og, b[0], warmup=1)
    eager_e = FlowTrainStep(me, oe)
    eager_e(*b[0])
    graphed(*b[1])
    eager_e(*b[1])
    FlowTrainStep(mg, og)(*b[2])  # an eager step on the graphed model's optimizer
    eager_e(*b[2])
    for o in (og, oe):
        o.param_groups[0]["lr"] = 5e-4  # plain assignment
    graphed(*b[1])
    eager_e(*b[1])
    for o in (og, oe):
        torch.optim.lr_scheduler.StepLR(o, step_size=1, gamma=0.5).step()  # 2.5e-4
    graphed(*b[2])
    eager_e(*b[2])
    torch.cuda.synchronize()
    worst = 0.0
    for (n, pg), pe in zip(mg.named_parameters(), me.parameters()):
        scale = float(pe.detach().abs().max()) + 1e-12
        worst = max(worst, float((pg - pe).abs().max()) / scale)
        sg, se = og.state.get(pg, {}).get("step"), oe.state.get(pe, {}).get("step")
        assert (sg is None) == (se is None), n
        if sg is not None:
            assert float(sg) == float(se) == 5.0, (n, float(sg), float(se))
    # the LR tensor (graph) and the float LR (eager) round 5e-4 / 2.5e-4 differently; a stale
    # LR or a stale bias correction would be off by ~1e-4 of the parameter scale
    assert worst < 2e-6, worst


def test_reductions_replay_from_graph():
    """The step's reductions replayed from a captured HIP graph equal their eager values on
    new data: torch's multi-block sum / mean / norm (loss and BN-statistics shapes) and the
    fixed-order dense.fixed_sum.  (Pins the claim in dense._FixedSum's docstring.)"""
    import dense
    x = torch.randn(8, 8192, 64, device=DEV)
    fns = {
        "sum_all": lambda t: t.sum(),
        "mean_all": lambda t: t.mean(),
        "norm_rows_mean": lambda t: torch.norm(t[..., :3], dim=2).sum(1).mean(),
        "sum_dim0_rows": lambda t: t.view(-1, 64).sum(0),
        "var_dim0_rows": lambda t: t.view(-1, 64).var(0, unbiased=False),
        "fixed_sum_all": lambda t: dense.fixed_sum(t),
        "fixed_sum_dim": lambda t: dense.fixed_sum(t.view(-1, 64), 0),
    }
    for f in fns.values():  # warm-up (lazy init) outside the capture
        f(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = {k: f(x) for k, f in fns.items()}
    bad = {}
    for seed in range(3):
        torch.manual_seed(100 + seed)
        x.copy_(torch.randn_like(x) * (seed + 1))
        g.replay()
        torch.cuda.synchronize()
        for k, f in fns.items():
            want = f(x)
            if not torch.equal(outs[k], want):
                bad[(seed, k)] = float((outs[k] - want).abs().max())
    assert not bad, bad


def test_coordinate_plan_equals_inline_searches():
    """PointConvBidirection.precompute_plan (FPS chain + the 13 coordinate-only kNN searches
    + their CSRs, the prefetched work of the training steps) gives the same flows, loss and
    gradients, bit for bit, as the forward running every search itself; an FPS-only plan
    (precompute_fps) as well."""
    import loss_functions as L
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(3)
    base = PointConvBidirection().to(DEV).train()
    p1, p2, fl = _batch(2, 8192, 51)
    plan = base.precompute_plan(p1, p2)
    nk = len(PointConvBidirection.PLAN_KNN)
    assert len(plan) == 4 + nk + sum((3 if k in PointConvBidirection._PLAN_RANKED else 2) +
                                     (5 if k in PointConvBidirection._PLAN_TILED else 0)
                                     for k in PointConvBidirection.PLAN_KNN)
    runs = []
    for pre in (None, base.precompute_fps(p1, p2), [t.clone() for t in plan]):
        m = copy.deepcopy(base)
        kw = {} if pre is None else {"fps_idx": pre}
        out = m(p1, p2, p1, p2, **kw)
        loss = L.multiScaleLoss(out[0], fl, out[1])
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach(), [f.detach() for f in out[0]],
                     {n: p.grad for n, p in m.named_parameters()}))
    ref = runs[0]
    for loss, flows, grads in runs[1:]:
        assert torch.equal(loss, ref[0]), (float(loss), float(ref[0]))
        for a, b in zip(flows, ref[1]):
            assert torch.equal(a, b)
        for n, g in grads.items():
            assert (g is None) == (ref[2][n] is None), n
            assert g is None or torch.equal(g, ref[2][n]), n


def test_coordinate_fork_is_bit_identical():
    """The decoder's flow-dependent searches and inverted indices on the side stream
    (models_bid_pointconv._CoordFork) give the same flows, loss and gradients, bit for bit, as
    running them in line: eager, under no_grad, and replayed from the captured train step."""
    import loss_functions as L
    import models_bid_pointconv as M
    from distill import graphed_flow_step, make_optimizer
    torch.manual_seed(4)
    base = M.PointConvBidirection().to(DEV).train()
    batches = [_batch(2, 8192, s) for s in (71, 72)]
    runs = []
    prev = M.COORD_FORK
    try:
        for on in (False, True):
            M.COORD_FORK = on
            m = copy.deepcopy(base)
            p1, p2, fl = batches[0]
            out = m(p1, p2, p1, p2)
            loss = L.multiScaleLoss(out[0], fl, out[1])
            loss.backward()
            with torch.no_grad():
                ev = m.eval()(p1, p2, p1, p2)[0]
            m.train()
            mg = copy.deepcopy(base)
            step = graphed_flow_step(mg, make_optimizer(mg, capturable=True), batches[0],
                                      warmup=1)
            gl = [float(step(*b)) for b in batches]
            torch.cuda.synchronize()
            runs.append((loss.detach(), [f.detach() for f in out[0]], [f for f in ev],
                         {n: p.grad for n, p in m.named_parameters()}, gl,
                         [p.detach().clone() for p in mg.parameters()]))
    finally:
        M.COORD_FORK = prev
    (l0, f0, e0, g0, gl0, p0), (l1, f1, e1, g1, gl1, p1_) = runs
    assert torch.equal(l0, l1), (float(l0), float(l1))
    for a, b in zip(f0 + e0, f1 + e1):
        assert torch.equal(a, b)
    for n, g in g1.items():
        assert (g is None) == (g0[n] is None), n
        assert g is None or torch.equal(g, g0[n]), n
    assert gl0 == gl1, (gl0, gl1)
    for a, b in zip(p0, p1_):
        assert torch.equal(a, b)


def test_teacher_stream_is_bit_identical():
    """The KD step's frozen-teacher forward on its own stream -- eagerly (distill._TeacherFork,
    beside the student's forward), graphed as a concurrent branch of the one step graph (the
    default) and graphed as a graph of its own beside the student's forward graph
    (TEACHER_GRAPH) -- gives the same losses and parameters, bit for bit, as running it in
    line.  (Before round 6 the two-stream forms disagreed now and then: packed f32
    instructions)"""
    import distill
    from distill import KDTrainStep, graphed_kd_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection as Net
    torch.manual_seed(1)
    teacher = Net().to(DEV)
    torch.manual_seed(2)
    base = Net().to(DEV)
    batches = [_batch(2, 4096, s) for s in (61, 62)]
    runs = []
    prev = distill.TEACHER_STREAM, distill.TEACHER_GRAPH
    try:
        for stream, graph in ((False, False), (True, False), (True, True)):
            distill.TEACHER_STREAM, distill.TEACHER_GRAPH = stream, graph
            m_e, m_g = copy.deepcopy(base), copy.deepcopy(base)
            eager = KDTrainStep(teacher, m_e, make_optimizer(m_e, capturable=True))
            graphed = graphed_kd_step(teacher, m_g, make_optimizer(m_g, capturable=True),
                                      batches[0], warmup=1)
            assert (graphed.graph_t is not None) == graph
            losses = [float(eager(*b)) for b in batches] + [float(graphed(*b)) for b in batches]
            torch.cuda.synchronize()
            runs.append((losses, [p.detach().clone() for p in m_e.parameters()],
                         [p.detach().clone() for p in m_g.parameters()]))
    finally:
        distill.TEACHER_STREAM, distill.TEACHER_GRAPH = prev
    l0, e0, g0 = runs[0]
    for l1, e1, g1 in runs[1:]:
        assert l0 == l1, (l0, l1)
        for a, b in zip(e0 + g0, e1 + g1):
            assert torch.equal(a, b)


def test_graphed_kd_steps_are_reproducible():
    """Two graphed KD steps built from identical models and replayed side by side on the same
    batches (configs[3]'s per-GPU slice, B=4, N=8192, the plan prefetched inside the graph,
    the teacher's forward a concurrent branch on its own stream) give the same loss and the
    same packed student gradients at every replay.  Before round 6
    they disagreed in about one replay in six and sometimes faulted: packed f32 instructions
    in the culled kNN gave wrong seed distances while the teacher's PointConv kernels ran
    beside them on the other stream (profiles/round06/race)."""
    from distill import graphed_kd_step, make_optimizer
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    torch.manual_seed(1)
    teacher = Teacher().to(DEV)
    torch.manual_seed(2)
    base = Student().to(DEV)
    batches = [_batch(4, 8192, s) for s in (81, 82, 83)]
    m1, m2 = copy.deepcopy(base), copy.deepcopy(base)
    g1 = graphed_kd_step(teacher, m1, make_optimizer(m1, capturable=True), batches[0], warmup=1)
    g2 = graphed_kd_step(teacher, m2, make_optimizer(m2, capturable=True), batches[0], warmup=1)
    for i in range(12):
        b, nxt = batches[i % 3], batches[(i + 1) % 3]
        l1 = g1(*b, next_batch=nxt)
        l2 = g2(*b, next_batch=nxt)
        torch.cuda.synchronize()
        assert torch.equal(l1, l2), (i, float(l1), float(l2))
        assert torch.equal(g1.G, g2.G), i
    for a, c in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, c)
