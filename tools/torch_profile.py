"""Attribute GPU time of one training step to torch ops and Python call sites.

    python tools/torch_profile.py [--batch 8] [--out gpurun_out/torch_prof.txt]

Runs a few warm-up steps of bench.py's FlowTrainStep, then profiles 2 steps with
torch.profiler (CUDA activity, Python stacks) and writes the top ops by device time,
grouped by op and by the innermost project call site.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import synthetic  # noqa: E402
from distill import FlowTrainStep, make_optimizer  # noqa: E402
from models_bid_pointconv import PointConvBidirection  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "torch_prof.txt"))
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PointConvBidirection().to(dev)
    opt = make_optimizer(model)
    step = FlowTrainStep(model, opt)
    p1, p2, fl = (torch.from_numpy(a).to(dev) for a in synthetic.ft3d_batch(args.batch, 8192, seed=3))
    for _ in range(3):
        step(p1, p2, fl)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        for _ in range(2):
            step(p1, p2, fl)
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        ka = prof.key_averages()
        f.write(ka.table(sort_by="self_device_time_total", row_limit=40, max_name_column_width=60))
        f.write("\n\n==== by input shape\n")
        f.write(prof.key_averages(group_by_input_shape=True).table(
            sort_by="self_device_time_total", row_limit=60, max_name_column_width=40,
            max_shapes_column_width=80))
        f.write("\n\n==== ops by input shape (self device us per step, calls per step)\n")
        shp = []
        for e in prof.key_averages(group_by_input_shape=True):
            t = getattr(e, "self_device_time_total", 0.0)
            if t > 0 and e.key.startswith("aten::"):
                shp.append((t / 2, e.count / 2, e.key, str(e.input_shapes)[:150]))
        shp.sort(reverse=True)
        for t, c, k, sh in shp[:150]:
            f.write(f"{t:9.1f} {c:6.1f} {k:28s} {sh}\n")
        f.write("\n\n==== by call site (self device us per step, calls per step, op, stack)\n")
        rows = []
        for e in prof.key_averages(group_by_stack_n=8):
            t = getattr(e, "self_device_time_total", 0.0)
            if t <= 0 or not e.key.startswith("aten::"):
                continue
            stack = [s for s in (e.stack or []) if "kd-pointcloud_amd" in s or "distill" in s]
            rows.append((t / 2, e.count / 2, e.key, " <- ".join(x.split("/")[-1] for x in stack[:4])))
        rows.sort(reverse=True)
        for t, c, k, st in rows[:120]:
            f.write(f"{t:9.1f} {c:6.1f} {k:28s} {st}\n")
        f.write("\n\n==== by call site, most launches first\n")
        rows.sort(key=lambda x: -x[1])
        for t, c, k, st in rows[:120]:
            f.write(f"{t:9.1f} {c:6.1f} {k:28s} {st}\n")
    print("wrote", args.out)


if __name__ == "__main__":
    main()
