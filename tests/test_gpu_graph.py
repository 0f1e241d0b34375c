"""The HIP-graph training step (distill.GraphedStep) performs exactly the eager step: same
kernels, same order, so parameters after a few steps agree bit for bit."""
import copy
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(b, n, seed):
    import synthetic
    return tuple(torch.from_numpy(a).to(DEV) for a in synthetic.ft3d_batch(b, n, seed=seed))


@pytest.mark.parametrize("mode", ["train", "kd", "kd_inline", "kd_tgraph", "kd_fork",
                                  "kd_fork_own"])
def test_graphed_step_equals_eager(mode, monkeypatch):
    """kd: the KD step as one graph with the teacher's forward a concurrent branch on the
    teacher stream (the default) against the eager KDTrainStep with the teacher on its own
    stream; kd_inline: the teacher in line (TEACHER_STREAM = False), graphed and eager;
    kd_tgraph: the teacher's forward as a graph of its own beside the student's forward graph,
    then loss + backward + Adam (TEACHER_GRAPH, distill.GraphedStep stages); kd_fork: the KD
    student keeps its decoder
    coordinate fork (models_bid_pointconv._CoordFork) on the parameter-gradient stream inside
    the student's forward graph; kd_fork_own: on a stream of its own (the round-3 capture_end
    segfault case)."""
    import distill
    import models_bid_pointconv
    from distill import (FlowTrainStep, KDTrainStep, graphed_flow_step, graphed_kd_step,
                         make_optimizer)
    from models_bid_pointconv import PointConvBidirection
    if mode.startswith("kd_fork"):
        monkeypatch.setattr(distill, "KD_COORD_FORK", True)
        monkeypatch.setattr(models_bid_pointconv, "SHARED_SIDE_STREAM", mode == "kd_fork")
        mode = "kd"
    if mode == "kd_inline":
        monkeypatch.setattr(distill, "TEACHER_GRAPH", False)
        monkeypatch.setattr(distill, "TEACHER_STREAM", False)
        mode = "kd"
    if mode == "kd_tgraph":
        monkeypatch.setattr(distill, "TEACHER_GRAPH", True)
        monkeypatch.setattr(distill, "TEACHER_STREAM", True)
        mode = "kd"
    torch.manual_seed(0)
    base = PointConvBidirection().to(DEV)
    teacher = PointConvBidirection().to(DEV) if mode == "kd" else None
    batches = [_batch(2, 2048, s) for s in (1, 2, 3)]
    eager_model = copy.deepcopy(base)
    graph_model = copy.deepcopy(base)
    opt_e = make_optimizer(eager_model, capturable=True)
    opt_g = make_optimizer(graph_model, capturable=True)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        if mode == "kd":
            eager = KDTrainStep(teacher, eager_model, opt_e)
            graphed = graphed_kd_step(teacher, graph_model, opt_g, batches[0], warmup=1)
        else:
            eager = FlowTrainStep(eager_model, opt_e)
            graphed = graphed_flow_step(graph_model, opt_g, batches[0], warmup=1)
    # a leftover warm-up autograd graph makes the captured backward's AccumulateGrad nodes
    # run on the warm-up stream (round-1 GPUTEST warning): capture must not see any
    stream_warn = [str(w.message) for w in caught if "AccumulateGrad" in str(w.message)
                   or "stream" in str(w.message).lower()]
    assert not stream_warn, stream_warn
    # the graphed step's constructor ran one eager warm-up step on batches[0]
    eager(*batches[0])
    losses = []
    # batches[1] -> batches[2] prefetched inside graph A; then batches[1] again, which the
    # previous replay did not prefetch (batches[2] was announced as next: eager recompute)
    seq = [(batches[1], batches[2]), (batches[2], batches[0]), (batches[1], None),
           (batches[2], None)]
    for b, nxt in seq:
        le = eager(*b)
        lg = graphed(*b, next_batch=nxt)
        losses.append((float(le), float(lg)))
    torch.cuda.synchronize()
    for le, lg in losses:
        assert le == lg, losses
    for (n, pe), pg in zip(eager_model.named_parameters(), graph_model.parameters()):
        assert torch.equal(pe, pg), n


def test_fps_prefetch_equals_inline():
    """FlowTrainStep with the next batch's FPS issued on a side stream gives the same losses
    and parameters as computing FPS inside the forward."""
    from distill import FlowTrainStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    base = PointConvBidirection().to(DEV)
    batches = [_batch(2, 2048, s) for s in (4, 5, 6)]
    m1, m2 = copy.deepcopy(base), copy.deepcopy(base)
    s1, s2 = FlowTrainStep(m1, make_optimizer(m1)), FlowTrainStep(m2, make_optimizer(m2))
    l1 = [float(s1(*b)) for b in batches]
    l2 = [float(s2(*b, next_batch=batches[i + 1] if i + 1 < len(batches) else None))
          for i, b in enumerate(batches)]
    assert l1 == l2, (l1, l2)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n


def test_eager_step_after_capture_has_no_stream_mismatch():
    """bench.py runs eager steps on the graphed model after the timed region (per-kernel
    roofline): the captured autograd graph must not outlive the capture, or those steps reuse
    its AccumulateGrad nodes (bound to the capture stream) -- the round-2 bench warning."""
    from distill import FlowTrainStep, graphed_flow_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    model = PointConvBidirection().to(DEV)
    opt = make_optimizer(model, capturable=True)
    b = _batch(2, 2048, 7)
    graphed = graphed_flow_step(model, opt, b, warmup=1)
    graphed(*b)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        FlowTrainStep(model, opt)(*b)
        torch.cuda.synchronize()
    bad = [str(w.message) for w in caught if "AccumulateGrad" in str(w.message)]
    assert not bad, bad


def test_parameter_gradient_stream_is_bit_identical():
    """wgrad.py: the parameter gradients issued on their own stream (PointConv weight kernel,
    dense split-K weight GEMMs, bias column sums) give the same parameters after two eager
    training steps, bit for bit, as issuing them in line; `.grad` is complete when
    backward() returns (read straight after it, no synchronisation)."""
    import wgrad
    from distill import FlowTrainStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    import loss_functions as L
    torch.manual_seed(0)
    base = PointConvBidirection().to(DEV)
    batches = [_batch(2, 4096, s) for s in (11, 12)]
    runs = []
    prev = wgrad.enabled
    try:
        for on in (False, True):
            wgrad.enabled = on
            m = copy.deepcopy(base)
            opt = make_optimizer(m)
            step = FlowTrainStep(m, opt)
            for b in batches:
                step(*b)
            out = m(*batches[0][:2], *batches[0][:2])
            loss = L.multiScaleLoss(out[0], batches[0][2], out[1])
            loss.backward()
            grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
            runs.append(({n: p.detach().clone() for n, p in m.named_parameters()}, grads))
    finally:
        wgrad.enabled = prev
    (p0, g0), (p1, g1) = runs
    for n in p0:
        assert torch.equal(p0[n], p1[n]), n
    assert g0.keys() == g1.keys()
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n


def test_parameter_gradient_stream_survives_in_place_gradient_accumulation():
    """A residual add around a dense layer: AddBackward hands the SAME gradient tensor to the
    layer's backward (whose weight gradient reads it on the side stream) and to the input
    buffer of the residual branch, which then adds the layer's input gradient into it -- in
    place whenever that buffer holds the only reference.  wgrad.run keeps the
    side-stream inputs referenced until the end-of-backward join, so the weight / bias
    gradients equal the in-line ones bit for bit.  The side stream is kept busy first (a long
    GEMM chain) so that an unprotected read would come after the in-place add."""
    import dense
    import wgrad
    torch.manual_seed(3)
    x0 = torch.randn(65536, 64, device=DEV)
    w1 = torch.randn(64, 64, device=DEV) * 0.1
    w2 = torch.randn(64, 64, device=DEV) * 0.1
    b2 = torch.randn(64, device=DEV) * 0.1
    big = torch.randn(2048, 2048, device=DEV)
    res = []
    prev = wgrad.enabled
    try:
        for on in (False, True):
            wgrad.enabled = on
            a = w1.clone().requires_grad_(True)
            w = w2.clone().requires_grad_(True)
            b = b2.clone().requires_grad_(True)
            h = dense.linear(x0, a)
            out = dense.linear(h, w, b) + h
            if on:  # queue work ahead on every side stream
                for sd in wgrad.side_streams(torch.device(DEV)):
                    sd.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(sd):
                        y = big
                        for _ in range(20):
                            y = y @ big * 1e-3
            (out * out).sum().backward()
            torch.cuda.synchronize()
            res.append([t.grad.clone() for t in (a, w, b)])
    finally:
        wgrad.enabled = prev
    for n, g0, g1 in zip(("w1", "w2", "b2"), *res):
        assert torch.equal(g0, g1), n


def test_parameter_gradient_stream_accumulates_onto_existing_grads():
    """Two backward() calls without zero_grad (gradient accumulation): the second pass's
    AccumulateGrad adds onto the first pass's .grad on the backward's stream, so wgrad.run
    must order those layers' side-stream kernels before it.  Bit-identical to
    issuing the parameter gradients in line."""
    import wgrad
    from models_bid_pointconv import PointConvBidirection
    import loss_functions as L
    torch.manual_seed(0)
    base = PointConvBidirection().to(DEV)
    batches = [_batch(2, 4096, s) for s in (21, 22)]
    runs = []
    prev = wgrad.enabled
    try:
        for on in (False, True):
            wgrad.enabled = on
            m = copy.deepcopy(base).train()
            for b in batches:  # no zero_grad in between
                out = m(*b[:2], *b[:2])
                L.multiScaleLoss(out[0], b[2], out[1]).backward()
            runs.append({n: p.grad.clone() for n, p in m.named_parameters()
                         if p.grad is not None})
    finally:
        wgrad.enabled = prev
    g0, g1 = runs
    assert g0.keys() == g1.keys()
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n


def test_capture_joins_forked_side_streams():
    """distill._join_capture_streams: work left unjoined on one of the process's side streams
    (here the KD teacher's stream) at the end of a captured step is joined into the capture
    stream before capture_end -- an unjoined capture crashes this runtime's capture_end
    instead of raising (tools/hip_capture_repro.hip `unjoined`) -- and the graph replays it."""
    import distill
    from distill import GraphedStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    import loss_functions as L
    torch.manual_seed(0)
    model = PointConvBidirection().to(DEV).train()
    opt = make_optimizer(model, capturable=True)
    b = _batch(1, 1024, 31)
    dev = torch.device(DEV, torch.cuda.current_device())
    side = distill._teacher_streams.get(dev.index)
    if side is None:
        side = distill._teacher_streams[dev.index] = torch.cuda.Stream(device=dev)
    marks = torch.zeros(4, device=DEV)

    def run(pos1, pos2, flow):
        out = model(pos1, pos2, pos1, pos2)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            marks.add_(1.0)  # never joined by this function
        return L.multiScaleLoss(out[0], flow, out[1])
    step = GraphedStep(run, model.parameters(), opt, b, warmup=1)
    torch.cuda.synchronize()
    before = float(marks[0])
    for _ in range(3):
        step(*b)
    torch.cuda.synchronize()
    assert float(marks[0]) == before + 3.0
