#!/usr/bin/env python
"""Headline benchmark: scene-flow pairs/sec, fwd+bwd, N=8192 (BASELINE.json `metric`).

One step = one training iteration of PointConvBidirection on B synthetic
FlyingThings3D-shaped pairs per GPU (BASELINE.json configs[2]: B=8, N=8192): forward,
multiScaleLoss, backward, Adam step (`--mode kd` adds the frozen teacher forward and the
biDirection_loss_ht KD objective of configs[3]).  With N GPUs: one process per GPU, DDP over
RCCL, per-GPU batch fixed (weak scaling), no data-path collective beyond DDP's gradient
all-reduce.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` is measured live over the timed region: every
launch of the chosen kernel is bracketed by HIP events on its stream, and its algorithmic
bytes (or flops) per launch are summed by the op wrapper.  `cpu_baseline` is the oracle's
pure-PyTorch CPU restatement of the reference path (square_distance+topk kNN,
torch.gather indexing, FPS replaced by a random subsample) on a bounded sample, rank 0 only.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3  # dense f32 MFMA peak (MI355X_MICROARCH.md, F32 row)
FP32_VALU_PEAK_TF = 157.3

# C entry point -> (bound, unit, peak, HIP kernels it launches).  An entry point is the unit
# the live timer brackets; tools/roofline_check.py sums the listed kernels' rocprofv3
# durations per entry launch to cross-check the live average.
ROOFLINE = {
    "kdpc_pointconv_bwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                           # first name: one launch per entry call (tools count launches by it)
                           ["pc_csr_sum_kernel", "pc_bwd_data_kernel", "pc_bwd_data_pipe_kernel",
                            "pc_bwd_weight_kernel", "pc_slab_sum_kernel", "pc_swizzle_bwd_kernel"]),
    "kdpc_pointconv_fwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                           ["pc_fwd_kernel", "pc_slab_sum_kernel"]),
    "kdpc_group_rows": ("hbm", "GB/s", HBM_PEAK_GBS, ["group_rows_kernel"]),
    "kdpc_group_points": ("hbm", "GB/s", HBM_PEAK_GBS, ["group_points_lds_kernel",
                                                         "group_points_kernel"]),
    "kdpc_knn_point": ("valu", "TFLOP/s", FP32_VALU_PEAK_TF, ["knn_kernel"]),
    "kdpc_cost_volume_fwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF, ["cost_volume_fwd_kernel"]),
    "kdpc_cost_volume_bwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF, ["cost_volume_bwd_kernel"]),
    "kdpc_idw_blend_fwd": ("hbm", "GB/s", HBM_PEAK_GBS, ["idw_fwd_kernel"]),
}
# the step's dominant entry point (rocprofv3 step profile, profiles/); the gather-bound
# grouping_operation the north star names is measured by gather_roofline()
PRIMARY_KERNEL = "kdpc_pointconv_bwd"
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU")
    ap.add_argument("--npoints", type=int, default=8192)
    ap.add_argument("--mode", choices=["train", "kd"], default="train")
    ap.add_argument("--roofline-kernel", default=PRIMARY_KERNEL)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="issue the step eagerly from Python (DDP for N>1) instead of replaying "
                         "it from HIP graphs (distill.GraphedStep, the default since round 2: "
                         "the eager step needs ~21 ms of host time per step, as much as the "
                         "GPU, and the graph replay carries the next batch's FPS chain on a "
                         "forked stream like the eager FpsPrefetch)")
    ap.add_argument("--graph", action="store_true", help="(default; kept for old command lines)")
    ap.add_argument("--measure-steps", type=int, default=2,
                    help="eager steps after the timed region for the per-kernel roofline")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle CPU path on a bounded sample: B=1 pair, N=npoints, fwd+bwd+Adam (--mode kd:
    frozen teacher fwd + student fwd+bwd + biDirection_loss_ht + Adam)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_model as M
    import synthetic
    torch.manual_seed(0)
    M.FPS_MODE["mode"] = "random"
    M.FPS_MODE["generator"] = torch.Generator().manual_seed(0)
    model = M.PointConvBidirection().train()
    teacher = M.PointConvBidirection().eval() if args.mode == "kd" else None
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    p1, p2, fl = (torch.from_numpy(a) for a in synthetic.ft3d_batch(1, args.npoints, seed=99))

    def step():
        out = model(p1, p2, p1, p2)
        if teacher is None:
            loss = M.multiScaleLoss(out[0], fl, out[1])
        else:
            with torch.no_grad():
                t = teacher(p1, p2, p1, p2)
            loss = M.biDirection_loss_ht(out[0], out[5], out[6], out[1], out[2], fl, t[0], t[5],
                                         t[6], t[1], t[2], 0.3, 0.8, layer=3)
        loss.backward()
        opt.step()
        opt.zero_grad()

    step()  # warm-up
    times = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(1.0 / med, 4), "unit": "pairs/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"1 pair x N={args.npoints}, "
                      f"{'KD step (teacher fwd + ' if teacher is not None else ''}"
                      f"fwd+bwd+Adam{')' if teacher is not None else ''}, median of {args.cpu_steps} "
                      f"steps after 1 warm-up ({med:.2f} s/step); oracle/torch_model.py "
                      f"(square_distance+topk kNN, torch.gather, FPS->randperm); "
                      f"host os.cpu_count()={os.cpu_count()}"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes
    (tools/pmc_traffic.py; FETCH_SIZE and WRITE_SIZE in separate passes, FETCH_SIZE doubled
    per MI355X_MICROARCH.md §HBM), or None when that kernel was not measured."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get("entries", {}).get(kernel)
    return None if e is None else e.get("hbm_bytes_per_launch")


def gather_roofline(dev, iters=20):
    """The north star's gather target at BASELINE configs[1]: grouping_operation (reference
    (B,C,N) layout) at B=8, C=64, N=8192, S=2048, K=16 on FPS centres + ball_query(r=0.5)
    indices, timed with HIP events over `iters` back-to-back launches on the launch stream
    (single ~15 us launches cannot be bracketed individually: the event packets cost as
    much as the kernel).  Algorithmic bytes B*(4CN + 4SK + 4CSK)."""
    import kdpc_native as K
    import synthetic
    B, C, N, S, Kn = 8, 64, 8192, 2048, 16
    xyz = torch.from_numpy(synthetic.ft3d_batch(B, N, seed=7)[0]).to(dev)
    centres = K.group_rows(xyz, K.furthest_point_sampling(xyz, S))
    idx = K.ball_query(0.5, Kn, xyz, centres)
    feats = torch.randn(B, C, N, device=dev)
    for _ in range(3):
        K.group_points(feats, idx)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        K.group_points(feats, idx)
    e1.record(stream)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    nbytes = B * (4 * C * N + 4 * S * Kn + 4 * C * S * Kn)
    achieved = nbytes / (us * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("kdpc_group_points"),
            "kernel": "kdpc_group_points", "hip_kernels": ROOFLINE["kdpc_group_points"][3],
            "workload": "grouping_operation B=8 C=64 N=8192 S=2048 K=16 (configs[1]), "
                        f"{iters} back-to-back launches",
            "avg_launch_us": round(us, 2), "algorithmic_bytes_per_launch": nbytes}


def roofline(kernel, summ):
    """Live roofline of one C entry point from the HIP-event launch timer."""
    if not summ or summ["ms"] <= 0:
        return None
    bound, unit, peak, kernels = ROOFLINE.get(kernel, ("hbm", "GB/s", HBM_PEAK_GBS, []))
    per_launch_ms = summ["ms"] / summ["launches"]
    if unit == "GB/s":
        achieved = summ["bytes"] / (summ["ms"] * 1e-3) / 1e9
    else:
        achieved = summ["flops"] / (summ["ms"] * 1e-3) / 1e12
    return {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": pmc_traffic(kernel),
            "kernel": kernel, "hip_kernels": kernels, "launches": summ["launches"],
            "avg_launch_us": round(per_launch_ms * 1e3, 2),
            "algorithmic_bytes_per_launch": round(summ["bytes"] / summ["launches"]),
            "algorithmic_flops_per_launch": round(summ["flops"] / summ["launches"]),
            "traffic_source": os.path.relpath(PMC_FILE, ROOT) if os.path.exists(PMC_FILE) else None}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if os.environ.get("KDPC_BLAS"):
        torch.backends.cuda.preferred_blas_library(os.environ["KDPC_BLAS"])

    import kdpc_native
    import synthetic
    from distill import (FlowTrainStep, KDTrainStep, graphed_flow_step, graphed_kd_step,
                         make_optimizer, wrap_ddp)
    from models_bid_pointconv import PointConvBidirection

    # inputs resident in HBM before timing; a few distinct batches per rank, cycled
    nb = 4
    batches = []
    for i in range(nb):
        p1, p2, fl = synthetic.ft3d_batch(args.batch, args.npoints, seed=1000 + rank,
                                          first_pair=i * args.batch)
        batches.append(tuple(torch.from_numpy(a).to(dev) for a in (p1, p2, fl)))

    torch.manual_seed(0)
    student = PointConvBidirection().to(dev)
    teacher = None
    if args.mode == "kd":
        torch.manual_seed(1)
        teacher = PointConvBidirection().to(dev)
    graph = not args.eager
    if graph:
        if world > 1:  # replicas start identical (DDP does this broadcast at construction)
            for t in list(student.parameters()) + list(student.buffers()):
                dist.broadcast(t.data, 0)
        opt = make_optimizer(student, capturable=True)
        try:
            if args.mode == "kd":
                step = graphed_kd_step(teacher, student, opt, batches[0])
            else:
                step = graphed_flow_step(student, opt, batches[0])
        except RuntimeError as exc:  # capture refused on this runtime: measure the eager step
            if world == 1:
                raise
            print(f"rank {rank}: HIP-graph capture failed ({exc}); eager DDP step instead",
                  file=sys.stderr, flush=True)
            graph = False
            torch.cuda.synchronize()
    if graph:
        eager = (KDTrainStep(teacher, student, opt) if args.mode == "kd"
                 else FlowTrainStep(student, opt))
    else:
        model = wrap_ddp(student, dev)
        opt = make_optimizer(model)
        step = KDTrainStep(teacher, model, opt) if args.mode == "kd" else FlowTrainStep(model, opt)
        eager = step

    # the eager steps issue the next batch's FPS chain on a side stream (distill.FpsPrefetch)
    # (the graphed step does the same inside graph A, on a forked stream)
    nxt = lambda i: {"next_batch": batches[(i + 1) % nb]}  # noqa: E731
    for i in range(args.warmup):
        step(*batches[i % nb], **nxt(i))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(*batches[i % nb], **nxt(i))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # host enqueue time of one eager step: the Python/torch.ops time to issue it, measured
    # from an idle device (the step is GPU-bound while this stays below ms_per_step)
    host = []
    for i in range(2):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        eager(*batches[i % nb])
        host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
    host_ms = round(min(host) * 1e3, 3)

    # per-kernel roofline: HIP events around every launch of the named C entry points, over
    # eager replays of the same step after the timed region (a graph replay has no
    # per-launch host hook); kernel durations do not depend on how the launch was issued
    timer = kdpc_native.LaunchTimer([args.roofline_kernel])
    kdpc_native.set_launch_timer(timer)
    for i in range(args.measure_steps):
        eager(*batches[i % nb])
    torch.cuda.synchronize()
    kdpc_native.set_launch_timer(None)
    summary = timer.summary()
    roof = roofline(args.roofline_kernel, summary.get(args.roofline_kernel))
    roof_gather = gather_roofline(dev)

    pairs = world * args.batch * args.steps
    line = {
        "metric": "scene-flow pairs/sec fwd+bwd @ N=8192; EPE3D vs ref; 1/2/4/8 MI355X",
        "value": round(pairs / dt, 3), "unit": "pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic FlyingThings3D-shaped pairs (kd-pointcloud_amd/synthetic.py), "
                "random-init weights",
        "config": {"workload": "PointConvBidirection fwd+bwd+Adam (BASELINE configs[2])"
                   if args.mode == "train" else
                   "KD step: teacher fwd + student fwd+bwd + biDirection_loss_ht (configs[3])",
                   "model": "models_bid_pointconv.PointConvBidirection",
                   "batch_per_gpu": args.batch, "global_batch": world * args.batch,
                   "npoints": args.npoints, "parallelism": f"dp{world}",
                   "step": "hip-graph" if graph else "eager"},
        "host_enqueue_ms": host_ms,
        "roofline": roof,
        "roofline_gather": roof_gather,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
