"""Diagnostic (GPU): does a second replay of the captured forward+backward (graph A) give the
eager result, with and without eager work between the replays?"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402


def batch(b, n, seed):
    import synthetic
    return tuple(torch.from_numpy(a).cuda() for a in synthetic.ft3d_batch(b, n, seed=seed))


def eager_loss(model, bt):
    import loss_functions
    m = copy.deepcopy(model)
    for p in m.parameters():
        p.grad = None
    m.train()
    flows, fps1, *_ = m(bt[0], bt[1], bt[0], bt[1])
    loss = loss_functions.multiScaleLoss(flows, bt[2], fps1)
    loss.backward()
    return float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}


def run(drop, interleave):
    import distill
    from distill import graphed_flow_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    distill.GraphedStep.drop_warmup_graph = drop
    torch.manual_seed(0)
    gm = PointConvBidirection().cuda()
    batches = [batch(2, 2048, s) for s in (1, 2, 3)]
    og = make_optimizer(gm, capturable=True)
    g = graphed_flow_step(gm, og, batches[0], warmup=1)
    other = PointConvBidirection().cuda()
    res = []
    for i, bt in enumerate(batches[1:]):
        want, wgrads = eager_loss(gm, bt)
        if interleave:  # unrelated eager work between replays
            eager_loss(other, batches[0])
        for s, t in zip(g.static, bt):
            s.copy_(t)
        g.graph_a.replay()
        torch.cuda.synchronize()
        bad = [(n, float((p.grad - wgrads[n]).abs().max()), p.grad._base is not None,
                p.grad.untyped_storage().nbytes() // 4, p.grad.numel())
               for n, p in gm.named_parameters() if n in wgrads and not torch.equal(p.grad, wgrads[n])]
        res.append((want, float(g.loss), bad))
        g.graph_b.replay()
    print(f"drop={drop} interleave={interleave}: (eager, graph, #grads differing) per replay {res}",
          flush=True)


run(True, False)
run(True, True)
