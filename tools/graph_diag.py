"""Diagnostic (GPU): is the captured loss tensor's storage overwritten by graph B, or by
work between replays?"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402


def batch(b, n, seed):
    import synthetic
    return tuple(torch.from_numpy(a).cuda() for a in synthetic.ft3d_batch(b, n, seed=seed))


def main(mode):
    from distill import graphed_kd_step, graphed_flow_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    gm = PointConvBidirection().cuda()
    teacher = PointConvBidirection().cuda()
    batches = [batch(2, 2048, s) for s in (1, 2, 3, 4)]
    og = make_optimizer(gm, capturable=True)
    if mode == "kd":
        g = graphed_kd_step(teacher, gm, og, batches[0], warmup=1)
    else:
        g = graphed_flow_step(gm, og, batches[0], warmup=1)
    for i, bt in enumerate(batches[1:]):
        for s, t in zip(g.static, bt):
            s.copy_(t)
        g.graph_a.replay()
        torch.cuda.synchronize()
        l1 = float(g.loss)
        if g.graph_b is not None:
            g.graph_b.replay()
        torch.cuda.synchronize()
        l2 = float(g.loss)
        g.graph_a.replay()  # replay A again with the updated parameters? no: same inputs
        torch.cuda.synchronize()
        l3 = float(g.loss)
        print(mode, i, "after A", l1, "after B", l2, "A again", l3, flush=True)
        if g.graph_b is not None:
            g.graph_b.replay()


main("kd")
main("train")
