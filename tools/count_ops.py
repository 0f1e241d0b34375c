"""Diagnostic (GPU): which CSR builds / colsums / torch kernels one training step issues.
usage: python tools/count_ops.py [B] [N]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402


def main(b=8, n=8192):
    import kdpc_native as K
    import synthetic
    from distill import FlowTrainStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    log = collections.Counter()
    orig_init = K.Csr.__init__

    def init(self, idx2d, nn):
        site = [f for f in traceback.extract_stack()[:-2] if "kd-pointcloud_amd" in f.filename][-2:]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in site)
        u = int(torch.unique(idx2d[0]).numel()) == idx2d.shape[1]
        log[("csr", tuple(idx2d.shape), nn, "unique" if u else "dup", where)] += 1
        orig_init(self, idx2d, nn)
    K.Csr.__init__ = init
    orig_cs = K.colsum

    def colsum(x2):
        site = [f for f in traceback.extract_stack()[:-1] if "kd-pointcloud_amd" in f.filename][-2:]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in site)
        log[("colsum", tuple(x2.shape), where)] += 1
        return orig_cs(x2)
    K.colsum = colsum
    dev = torch.device("cuda")
    p1, p2, fl = (torch.from_numpy(a).to(dev) for a in synthetic.ft3d_batch(b, n, seed=1))
    torch.manual_seed(0)
    model = PointConvBidirection().to(dev)
    step = FlowTrainStep(model, make_optimizer(model))
    step(p1, p2, fl)
    torch.cuda.synchronize()
    log.clear()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        step(p1, p2, fl)
        torch.cuda.synchronize()
    for k, v in sorted(log.items(), key=lambda kv: str(kv[0])):
        print(v, k)
    print(prof.key_averages().table(sort_by="count", row_limit=45))
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof2:
        step(p1, p2, fl)
        torch.cuda.synchronize()
    print(prof2.key_averages().table(sort_by="self_cuda_time_total", row_limit=70,
                                     max_name_column_width=60))
    print(prof2.key_averages(group_by_stack_n=0).table(sort_by="cuda_time_total", row_limit=40,
                                                       max_name_column_width=60))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
