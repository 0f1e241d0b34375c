"""Per-entry-point rooflines of the training step (GPU): every C entry point of bench.ROOFLINE
timed with HIP events over eager steps (kdpc_native.LaunchTimer, as bench.py's live roofline),
its algorithmic bytes / flops per launch, and -- when profiles/pmc_traffic.json holds the
entry -- the counter HBM bytes per launch against the algorithmic ones.

    python tools/entry_rooflines.py [--steps 2] [--json profiles/roundNN/entry_rooflines.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kd-pointcloud_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--npoints", type=int, default=8192)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    import bench
    import kdpc_native
    import synthetic
    from distill import FlowTrainStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PointConvBidirection().to(dev).train()
    step = FlowTrainStep(model, make_optimizer(model))
    batches = [tuple(torch.from_numpy(a).to(dev) for a in
                     synthetic.ft3d_batch(args.batch, args.npoints, seed=s)) for s in (1, 2)]
    for i in range(2):
        step(*batches[i % 2])
    torch.cuda.synchronize()
    # a ~100 us GPU spin before each bracketed launch: the eager step is host-bound, and the
    # spin lets the host enqueue the whole entry before its start event fires
    timer = kdpc_native.LaunchTimer(list(bench.ROOFLINE), lead_cycles=250000)
    kdpc_native.set_launch_timer(timer)
    for i in range(args.steps):
        step(*batches[i % 2])
    torch.cuda.synchronize()
    kdpc_native.set_launch_timer(None)
    summ = timer.summary()
    wl = bench.workload_key("train", args.batch, args.npoints)
    out = {"workload": f"PointConvBidirection train step B={args.batch} N={args.npoints}, "
                       f"{args.steps} eager steps", "entries": {}}
    for name, (bound, unit, peak, kernels) in bench.ROOFLINE.items():
        s = summ.get(name)
        if not s:
            continue
        r = bench.roofline_obj(name, wl, s["ms"], s["launches"], s["bytes"], s["flops"])
        alg = r["algorithmic_bytes_per_launch"]
        if r["traffic"] is not None and alg:
            r["traffic_over_algorithmic"] = round(r["traffic"] / alg, 3)
        r["launches_per_step"] = s["launches"] / args.steps
        r["ms_per_step"] = round(s["ms"] / args.steps, 3)
        out["entries"][name] = r
        print(f"{name:28s} {r['avg_launch_us']:9.1f} us x {r['launches_per_step']:4.1f}/step  "
              f"{r['achieved']:8.1f} {unit} = {r['frac']:.3f} of {peak}  traffic/alg "
              f"{r.get('traffic_over_algorithmic')}", flush=True)
    if args.json:
        os.makedirs(os.path.dirname(os.path.abspath(args.json)), exist_ok=True)
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
