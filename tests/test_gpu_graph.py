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


@pytest.mark.parametrize("mode", ["train", "kd"])
def test_graphed_step_equals_eager(mode):
    from distill import (FlowTrainStep, KDTrainStep, graphed_flow_step, graphed_kd_step,
                         make_optimizer)
    from models_bid_pointconv import PointConvBidirection
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
