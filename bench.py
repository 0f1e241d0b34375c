#!/usr/bin/env python
"""Headline benchmark: scene-flow pairs/sec, fwd+bwd, N=8192 (BASELINE.json `metric`).

One step = one training iteration of PointConvBidirection on B synthetic
FlyingThings3D-shaped pairs per GPU (BASELINE.json configs[2]: B=8, N=8192): forward,
multiScaleLoss, backward, Adam step.  With N GPUs: one process per GPU, per-GPU batch fixed
(weak scaling); the only collective is the gradient all-reduce (bucketed, overlapped with
the backward: distill.GraphedStep).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Besides the headline (configs[2]) it carries sub-records:
  kd_step         configs[3]'s per-GPU slice: the KD step (teacher fwd + student fwd/bwd +
                  biDirection_loss_ht + Adam) at B=4 per GPU, its own timed region, roofline
                  and CPU baseline (every N: at N=8 it is configs[3]'s B=32 over 8 GPUs);
  configs1        configs[1] microbench (N=1): FPS, ball_query, grouping_operation, gather;
  roofline_knn    configs[4] (N=1): culled kNN K=32 at N=65536, B=4;
  step_roofline   the whole step against the model's algorithmic flops / bytes.
`roofline` objects are measured live: HIP events on the launch stream around the timed
launches, algorithmic bytes (or flops) per launch from SURVEY §8d.  `traffic` is the PMC
HBM bytes per launch from profiles/pmc_traffic.json for the SAME (workload, entry) only,
else null.  `cpu_baseline` is the oracle's pure-PyTorch CPU restatement of the reference
path (square_distance+topk kNN, torch.gather indexing, FPS replaced by a random subsample)
on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3  # dense f32 MFMA peak (MI355X_MICROARCH.md, F32 row)
# The PointConv kernels run their f32 GEMMs as six bf16 MFMAs per product (three-plane split,
# f32-accurate): their own ceiling is the dense bf16 rate / 6 (2.52 PF: 32 cycles
# per 32x32x16 MFMA per SIMD at 2.4 GHz), reported beside the f32 peak the roofline keeps.
SPLIT_BF16_PEAK_TF = round(2 * 32 * 32 * 16 / 32 * 1024 * 2.4e9 / 1e12 / 6, 1)
SPLIT_BF16_ENTRIES = ("kdpc_pointconv_bwd", "kdpc_pointconv_fwd")
FP32_VALU_PEAK_TF = 157.3  # f32 vector peak (same table)

# C entry point -> (bound, unit, peak, HIP kernels it launches).  An entry point is the unit
# the live timer brackets; tools/roofline_check.py sums the listed kernels' rocprofv3
# durations per entry launch to cross-check the live average.
ROOFLINE = {
    "kdpc_pointconv_bwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                           # first name: one launch per entry call (tools count launches by it)
                           ["pc_csr_sum_kernel", "pc_swizzle_bwd3_kernel",
                            "pc_bwd_data_kernel",
                            "pc_bwd_data_pipe_kernel", "pc_bwd_weight_kernel",
                            "pc_bwd_weight_x6_kernel", "pc_slab_sum_kernel"]),
    "kdpc_pointconv_fwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                           ["pc_fwd_kernel", "pc_swizzle_fwd3_kernel", "pc_slab_sum_kernel"]),
    "kdpc_group_rows": ("hbm", "GB/s", HBM_PEAK_GBS, ["group_rows_kernel"]),
    "kdpc_group_points": ("hbm", "GB/s", HBM_PEAK_GBS, ["group_points_lds_kernel",
                                                         "group_points_kernel",
                                                         "transpose_cn_kernel",
                                                         "group_points_pm_kernel"]),
    # kNN: plain scan (knn_kernel) or the culled scan (ref_sort / query_sort / chunk boxes /
    # knn_cull); work = brute-force-equivalent distance evaluations (8 flops each), bytes =
    # B*(12Nq + 12Nr + 4*Nq*K)
    "kdpc_knn_point": ("hbm", "GB/s", HBM_PEAK_GBS,
                       ["ref_sort_kernel", "query_sort_kernel", "chunk_box_kernel",
                        "knn_cull_kernel", "knn_kernel"]),
    "kdpc_gather_points": ("hbm", "GB/s", HBM_PEAK_GBS, ["gather_points_lds_kernel",
                                                          "gather_points_kernel"]),
    # cost volume, D <= 64 (cost_volume.hip) and the wide levels D in {128, 256} (the one-kernel
    # MFMA path of cost_volume_wide.hip) as separate entries (kdpc_native labels them by D)
    "kdpc_cost_volume_fwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF, ["cost_volume_fwd_kernel"]),
    "kdpc_cost_volume_fwd_wide": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                                  ["cvw_fused_fwd_kernel"]),
    "kdpc_cost_volume_bwd": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF, ["cost_volume_bwd_kernel"]),
    # the model's backward: rows in CSR order + contiguous per-point sums (+ the slab colsum)
    "kdpc_cost_volume_bwd_csr": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                                 ["cost_volume_bwd_kernel", "cv_rows_sum_lds_kernel<32>",
                                  "cv_rows_sum_lds_kernel<64>"]),
    "kdpc_cost_volume_bwd_csr_wide": ("mfma", "TFLOP/s", FP32_MFMA_PEAK_TF,
                                      ["cvw_fused_bwd_kernel", "cvw_transpose_kernel",
                                       "cv_rows_sum_lds_kernel<128>",
                                       "cv_rows_sum_lds_kernel<256>"]),
    "kdpc_idw_blend_fwd": ("hbm", "GB/s", HBM_PEAK_GBS, ["idw_fwd_kernel"]),
}
# the step's dominant entry point (rocprofv3 step profile, profiles/)
PRIMARY_KERNEL = "kdpc_pointconv_bwd"
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")
# per-pair algorithmic work of the whole model step: fwd+bwd dense flops and
# grouping traffic
STEP_FLOPS_PER_PAIR = 78.8e9
STEP_BYTES_PER_PAIR = 894e6


def workload_key(mode, batch, npoints):
    """The PMC workload key of a step section (profiles/pmc_traffic.json `workloads`)."""
    return f"{mode}_b{batch}_n{npoints}"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU (train step)")
    ap.add_argument("--kd-batch", type=int, default=4,
                    help="pairs per GPU of the KD step (configs[3]: 32 over 8 GPUs)")
    ap.add_argument("--npoints", type=int, default=8192)
    ap.add_argument("--mode", choices=["train", "kd"], default="train",
                    help="the headline step (kd: the KD step at --batch is the headline)")
    ap.add_argument("--sections", default="train,kd,configs1,knn",
                    help="comma list of train, kd, configs1, knn, gather_c3, gather_c64 "
                         "(PMC passes run one each)")
    ap.add_argument("--roofline-kernel", default=PRIMARY_KERNEL)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="issue the step eagerly from Python (DDP for N>1) instead of replaying "
                         "it from HIP graphs (distill.GraphedStep, the default: the eager step "
                         "needs about as much host time as the GPU needs)")
    ap.add_argument("--graph", action="store_true", help="(default; kept for old command lines)")
    ap.add_argument("--measure-steps", type=int, default=2,
                    help="eager steps after the timed region for the per-kernel roofline")
    return ap.parse_args(argv)


def _events(stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    return e0, e1


# ------------------------------------------------------------------ PMC / roofline helpers
def pmc_traffic(workload, entry):
    """HBM bytes per launch of `entry` measured by the committed rocprofv3 --pmc passes on the
    SAME workload (tools/pmc_traffic.py; FETCH_SIZE and WRITE_SIZE in separate passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), or None when that (workload, entry)
    was not measured."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get("workloads", {}).get(workload, {}).get("entries", {}).get(entry)
    return None if e is None else e.get("hbm_bytes_per_launch")


def roofline_obj(entry, workload, ms, launches, nbytes, flops, bound=None, **extra):
    """A roofline object from summed live launch times and summed algorithmic work."""
    if ms <= 0 or launches <= 0:
        return None
    b0, unit, peak, kernels = ROOFLINE.get(entry, ("hbm", "GB/s", HBM_PEAK_GBS, []))
    bound = bound or b0
    if bound == "hbm":
        unit, peak = "GB/s", HBM_PEAK_GBS
        achieved = nbytes / (ms * 1e-3) / 1e9
    else:
        achieved = flops / (ms * 1e-3) / 1e12
    out = {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
           "frac": round(achieved / peak, 4), "traffic": pmc_traffic(workload, entry),
           "kernel": entry, "hip_kernels": kernels, "workload": workload,
           "launches": launches, "avg_launch_us": round(ms / launches * 1e3, 2),
           "algorithmic_bytes_per_launch": round(nbytes / launches),
           "algorithmic_flops_per_launch": round(flops / launches),
           "traffic_source": os.path.relpath(PMC_FILE, ROOT)}
    if entry in SPLIT_BF16_ENTRIES and bound == "mfma":
        out["matrix_path"] = "f32 products as 6 bf16 MFMAs (three-plane split)"
        out["peak_split_bf16"] = SPLIT_BF16_PEAK_TF
        out["frac_split_bf16"] = round(achieved / SPLIT_BF16_PEAK_TF, 4)
    out.update(extra)
    return out


# ------------------------------------------------------------------------- CPU baseline
def cpu_baseline(args, mode):
    """Oracle CPU path on a bounded sample: B=1 pair, N=npoints, fwd+bwd+Adam (mode kd:
    frozen teacher fwd + student fwd+bwd + biDirection_loss_ht + Adam)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import synthetic
    import torch_model as M
    torch.manual_seed(0)
    M.FPS_MODE["mode"] = "random"
    M.FPS_MODE["generator"] = torch.Generator().manual_seed(0)
    model = M.PointConvBidirection().train()
    teacher = M.PointConvBidirection().eval() if mode == "kd" else None
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
    what = ("KD step (teacher fwd + student fwd+bwd + biDirection_loss_ht + Adam)"
            if teacher is not None else "fwd+multiScaleLoss+bwd+Adam")
    return {"value": round(1.0 / med, 4), "unit": "pairs/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"1 pair x N={args.npoints}, {what}, median of {args.cpu_steps} steps after "
                      f"1 warm-up ({med:.2f} s/step); oracle/torch_model.py "
                      f"(square_distance+topk kNN, torch.gather, FPS->randperm); "
                      f"host os.cpu_count()={os.cpu_count()}"}


# --------------------------------------------------------------------------- step section
def step_section(args, mode, batch, dev, world, rank):
    """Build the (graphed) train or KD step at `batch` pairs per GPU, time args.steps of it,
    then the live per-kernel roofline of args.roofline_kernel over eager replays."""
    import kdpc_native
    import synthetic
    from distill import (FlowTrainStep, KDTrainStep, graphed_flow_step, graphed_kd_step,
                         make_optimizer, wrap_ddp)
    from models_bid_pointconv import PointConvBidirection

    # inputs resident in HBM before timing; a few distinct batches per rank, cycled
    nb = 4
    batches = []
    for i in range(nb):
        p1, p2, fl = synthetic.ft3d_batch(batch, args.npoints, seed=1000 + rank,
                                          first_pair=i * batch)
        batches.append(tuple(torch.from_numpy(a).to(dev) for a in (p1, p2, fl)))

    torch.manual_seed(0)
    student = PointConvBidirection().to(dev)
    teacher = None
    if mode == "kd":
        torch.manual_seed(1)
        teacher = PointConvBidirection().to(dev)
    graph = not args.eager
    step_kind = "hip-graph"
    if graph:
        if world > 1:  # replicas start identical (DDP does this broadcast at construction)
            for t in list(student.parameters()) + list(student.buffers()):
                dist.broadcast(t.data, 0)
        opt = make_optimizer(student, capturable=True)

        def build(overlap=None):
            if mode == "kd":
                return graphed_kd_step(teacher, student, opt, batches[0], overlap=overlap)
            return graphed_flow_step(student, opt, batches[0], overlap=overlap)
        try:
            step = build()
        except RuntimeError as exc:  # RCCL capture refused: the serial multi-rank schedule
            if world == 1:
                raise
            print(f"rank {rank}: captured all-reduce failed ({exc}); serial schedule instead",
                  file=sys.stderr, flush=True)
            torch.cuda.synchronize()
            step = build(overlap=False)
        step_kind += step.schedule_name()
        eager = (KDTrainStep(teacher, student, opt) if mode == "kd"
                 else FlowTrainStep(student, opt))
    else:
        model = wrap_ddp(student, dev)
        opt = make_optimizer(model)
        step = KDTrainStep(teacher, model, opt) if mode == "kd" else FlowTrainStep(model, opt)
        eager = step
        step_kind = "eager" + (" ddp" if world > 1 else "")

    # the eager steps issue the next batch's FPS chain on a side stream (distill.FpsPrefetch);
    # the graphed step does the same inside its graph, on a forked stream
    nxt = lambda i: {"next_batch": batches[(i + 1) % nb]}  # noqa: E731
    for i in range(args.warmup):
        step(*batches[i % nb], **nxt(i))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(*batches[i % nb], **nxt(i))
    t_issue = time.perf_counter() - t0  # host time to issue the K steps (graph replays)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # host enqueue time of one eager step (Python / torch.ops issue time from an idle device)
    host = []
    for i in range(2):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        eager(*batches[i % nb])
        host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()

    # per-kernel roofline: HIP events around every launch of the entry point, over eager
    # replays of the same step after the timed region (a graph replay has no per-launch host
    # hook); kernel durations do not depend on how the launch was issued
    timer = kdpc_native.LaunchTimer([args.roofline_kernel], lead_cycles=250000)  # ~100 us
    kdpc_native.set_launch_timer(timer)
    # spin kernels bracket the window in a kernel trace (tools/roofline_check.py counts only
    # the launches between them: the graph replays run the entry's kernels concurrently with
    # the parameter-gradient stream, which lengthens them)
    torch.cuda.synchronize()
    torch.cuda._sleep(64)
    torch.cuda.synchronize()
    for i in range(args.measure_steps):
        eager(*batches[i % nb])
    torch.cuda.synchronize()
    torch.cuda._sleep(64)
    torch.cuda.synchronize()
    kdpc_native.set_launch_timer(None)
    s = timer.summary().get(args.roofline_kernel)
    wl = workload_key(mode, batch, args.npoints)
    roof = None if not s else roofline_obj(args.roofline_kernel, wl, s["ms"], s["launches"],
                                           s["bytes"], s["flops"])
    pairs = world * batch * args.steps
    ms = dt / args.steps * 1e3
    res = {"value": round(pairs / dt, 3), "unit": "pairs/s", "ms_per_step": round(ms, 3),
           "steps": args.steps, "warmup": args.warmup, "batch_per_gpu": batch,
           "global_batch": world * batch, "step": step_kind,
           "host_enqueue_ms": round(min(host) * 1e3, 3),
           "host_issue_ms_per_step": round(t_issue / args.steps * 1e3, 3),
           "roofline": roof,
           "step_roofline": {
               "bound": "mfma", "unit": "TFLOP/s", "peak": FP32_MFMA_PEAK_TF,
               "achieved": round(batch * STEP_FLOPS_PER_PAIR / (ms * 1e-3) / 1e12, 2),
               "frac": round(batch * STEP_FLOPS_PER_PAIR / (ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TF, 4),
               "hbm_frac": round(batch * STEP_BYTES_PER_PAIR / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
               "work_per_pair": "78.8 GFLOP dense fwd+bwd, 894 MB grouping traffic (SURVEY §8d)"
                                + (" + the teacher fwd (26.25 GFLOP, not counted)"
                                   if mode == "kd" else "")}}
    del step, eager, opt, student, teacher, batches
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


# ----------------------------------------------------------------------- microbenchmarks
def _time_launches(fn, iters, stream, warmup=3):
    for _ in range(warmup):
        fn()
    e0, e1 = _events(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters  # ms per launch


def _time_graph(fn, iters, warmup=3):
    """ms per launch of `iters` launches captured in one HIP graph and replayed: the GPU runs
    them back to back with no host issue in between (a ~3-5 us kernel issued from the host
    one by one measures the issue rate, not the kernel)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        for _ in range(iters):
            fn()
    for _ in range(10):  # ~thousands of launches first: clocks up, caches warm
        g.replay()
    torch.cuda.synchronize()
    times = []
    for _ in range(7):  # the median replay: robust to another process's burst on the GPU
        e0, e1 = _events(torch.cuda.current_stream())
        g.replay()
        e1.record(torch.cuda.current_stream())
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times)[3] / iters
    del g
    return ms


def _time_graph_rotated(fns, iters, warmup=1):
    """ms per launch of `iters` launches cycling over `fns` (each on its own inputs), captured
    in one HIP graph and replayed.  With the distinct inputs of the rotation totalling well
    over the 256 MiB Infinity Cache (MALL) plus the 8 x 4 MB of L2, every launch reads its
    inputs back from HBM: the cache-busting figure, where `_time_graph` on one
    input set measures the cache-resident one."""
    for f in fns:
        for _ in range(warmup):
            f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        for i in range(iters):
            fns[i % len(fns)]()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    times = []
    for _ in range(7):
        e0, e1 = _events(torch.cuda.current_stream())
        g.replay()
        e1.record(torch.cuda.current_stream())
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times)[3] / iters
    del g
    return ms


MALL_BYTES = 256 << 20  # MI355X Infinity Cache (MI355X_MICROARCH.md)


def configs1_section(dev):
    """BASELINE configs[1]: FPS + ball_query + grouping_operation (+ gather_operation) at
    B=8, N=8192, S=2048, K=16, C=64; indices bit-exact (tests/test_gpu_kernels.py).  Each op
    timed with HIP events on its launch stream over back-to-back launches (a single ~15 us
    launch cannot be bracketed alone: the event packets cost as much as the kernel)."""
    import kdpc_native as K
    import synthetic
    B, C, N, S, Kn = 8, 64, 8192, 2048, 16
    stream = torch.cuda.current_stream(dev)
    xyz = torch.from_numpy(synthetic.ft3d_batch(B, N, seed=7)[0]).to(dev)
    fps_ms = _time_launches(lambda: K.furthest_point_sampling(xyz, S), 5, stream)
    fidx = K.furthest_point_sampling(xyz, S)
    centres = K.group_rows(xyz, fidx)
    bq_ms = _time_launches(lambda: K.ball_query(0.5, Kn, xyz, centres), 20, stream)
    idx = K.ball_query(0.5, Kn, xyz, centres)
    feats = torch.randn(B, C, N, device=dev)
    wl = "configs1_b8_n8192_s2048_k16_c64"
    g_ms = _time_launches(lambda: K.group_points(feats, idx), 100, stream, warmup=10)
    g_bytes = B * (4 * C * N + 4 * S * Kn + 4 * C * S * Kn)
    # gather_operation: the model gathers xyz (C=3, index_points_gather); C=64 as well
    xyz_cn = xyz.permute(0, 2, 1).contiguous()
    # ~3-5 us launches: 200 of them replayed from one HIP graph
    ga3_ms = _time_graph(lambda: K.gather_points(xyz_cn, fidx), 200)
    ga64_ms = _time_graph(lambda: K.gather_points(feats, fidx), 200)
    ga_bytes = lambda c: B * (4 * c * N + 4 * S + 4 * c * S)  # noqa: E731
    # the same two ops rotated over distinct input sets (features + FPS / ball_query indices of
    # other clouds) whose bytes between two uses of one set exceed 2x the MALL: HBM figures
    nrot_g = 8   # 8 x 85 MB per grouping launch
    nrot_a = 32  # 32 x 21 MB per gather launch
    sets = []
    for r in range(max(nrot_g, nrot_a)):
        xr = torch.from_numpy(synthetic.ft3d_batch(B, N, seed=100 + r)[0]).to(dev)
        fr = K.furthest_point_sampling(xr, S)
        ir = K.ball_query(0.5, Kn, xr, K.group_rows(xr, fr)) if r < nrot_g else None
        sets.append((torch.randn(B, C, N, device=dev), fr, ir))
    gr_ms = _time_graph_rotated([lambda s=s: K.group_points(s[0], s[2]) for s in sets[:nrot_g]],
                                64)
    ar_ms = _time_graph_rotated([lambda s=s: K.gather_points(s[0], s[1]) for s in sets[:nrot_a]],
                                128)
    reuse_g = (nrot_g - 1) * g_bytes
    reuse_a = (nrot_a - 1) * ga_bytes(64)
    del sets
    return {
        "workload": "B=8 N=8192: FPS 8192->2048, ball_query r=0.5 K=16, grouping C=64 S=2048 "
                    "K=16, gather C=3 (the model's xyz) and C=64 (BASELINE configs[1])",
        "fps": {"us_per_call": round(fps_ms * 1e3, 2),
                "us_per_dependent_step": round(fps_ms * 1e3 / (S - 1), 4),
                "distance_updates_per_s": round(B * N * S / (fps_ms * 1e-3), 1),
                "bound": "latency (S-1 dependent block-wide argmax steps per cloud)"},
        "ball_query": {"us_per_call": round(bq_ms * 1e3, 2), "queries": B * S,
                       "bound": "latency (per-query serial scan with early exit)"},
        "grouping_operation": roofline_obj("kdpc_group_points", wl, g_ms, 1, g_bytes, 0),
        # PMC traffic keyed per channel count (the two launches differ 20x in bytes)
        "gather_operation_c3": roofline_obj("kdpc_gather_points", "configs1_gather_c3", ga3_ms, 1,
                                            ga_bytes(3), 0, bound="hbm", grid_workgroups=B * 3,
                                            note="1.0 MB per launch (24 rows of 32 KiB): "
                                                 "launch-latency-bound; timed as 200 "
                                                 "launches replayed from one HIP graph"),
        "gather_operation_c64": roofline_obj("kdpc_gather_points", "configs1_gather_c64",
                                             ga64_ms, 1, ga_bytes(64), 0, bound="hbm",
                                             grid_workgroups=B * 64,
                                             note="one input set replayed: cache-resident "
                                                  "(16.8 MB < 256 MiB MALL); the HBM figure is "
                                                  "gather_operation_c64_rotated"),
        # cache-busting figures: distinct inputs per launch, each set
        # re-read only after > 2x the MALL of other launches' traffic
        "grouping_operation_rotated": roofline_obj(
            "kdpc_group_points", wl + "_rot8", gr_ms, 1, g_bytes, 0, bound="hbm",
            rotation_sets=nrot_g, bytes_between_reuse=reuse_g,
            mall_bytes=MALL_BYTES, measured_hbm_ceiling_frac=0.79,
            note="64 launches over 8 distinct (features, ball_query idx) sets, one HIP graph"),
        "gather_operation_c64_rotated": roofline_obj(
            "kdpc_gather_points", "configs1_gather_c64_rot32", ar_ms, 1, ga_bytes(64), 0,
            bound="hbm", grid_workgroups=B * 64, rotation_sets=nrot_a,
            bytes_between_reuse=reuse_a, mall_bytes=MALL_BYTES, measured_hbm_ceiling_frac=0.79,
            note="128 launches over 32 distinct (features, FPS idx) sets, one HIP graph"),
    }


def gather_section(dev, c):
    """gather_operation alone at configs[1] (B=8, N=8192, M=2048) for C channels: the
    single-workload run the per-C PMC passes profile (sections gather_c3 / gather_c64)."""
    import kdpc_native as K
    import synthetic
    B, N, S = 8, 8192, 2048
    stream = torch.cuda.current_stream(dev)
    xyz = torch.from_numpy(synthetic.ft3d_batch(B, N, seed=7)[0]).to(dev)
    fidx = K.furthest_point_sampling(xyz, S)
    pts = (xyz.permute(0, 2, 1).contiguous() if c == 3 else torch.randn(B, c, N, device=dev))
    ms = _time_graph(lambda: K.gather_points(pts, fidx), 200)
    return roofline_obj("kdpc_gather_points", f"configs1_gather_c{c}", ms, 1,
                        B * (4 * c * N + 4 * S + 4 * c * S), 0, bound="hbm",
                        grid_workgroups=B * c)


def knn_section(dev):
    """BASELINE configs[4]: kNN K=32 at N=65536 per frame, B=4 (queries pc1, refs pc2), the
    culled scan (ref/query Morton sorts + chunk boxes + knn_cull), plus the grouping of C=32
    features by its indices."""
    import kdpc_native as K
    import synthetic
    B, N, Kn, C = 4, 65536, 32, 32
    stream = torch.cuda.current_stream(dev)
    p1, p2, _ = (torch.from_numpy(a).to(dev) for a in synthetic.ft3d_batch(B, N, seed=11))
    ms = _time_graph(lambda: K.knn_point(Kn, p2, p1), 5)  # its 4-5 kernels back to back
    idx = K.knn_point(Kn, p2, p1)
    # the distance evaluations the culled scan really issues (visited 64-ref chunks x 64 x
    # queries per wave + the 256-ref seed window per query), counted by the kernel in a
    # separate, untimed launch that returns the same indices
    idx_c, evals = K.knn_point_evals(Kn, p2, p1)
    assert torch.equal(idx_c, idx)
    nbytes = B * (12 * N + 12 * N + 4 * N * Kn)
    wl = "knn_b4_n65536_k32"
    brute = float(B) * N * N
    roof = roofline_obj("kdpc_knn_point", wl, ms, 1, nbytes, 8.0 * evals, bound="hbm",
                        evals_per_launch=evals,
                        evals_vs_brute_force=round(evals / brute, 5),
                        valu={"achieved_tflops": round(8.0 * evals / (ms * 1e-3) / 1e12, 3),
                              "peak": FP32_VALU_PEAK_TF,
                              "frac": round(8.0 * evals / (ms * 1e-3) / 1e12 / FP32_VALU_PEAK_TF,
                                            4),
                              "note": "8 flops per distance evaluation the culled scan issued "
                                      "(counted); the scan is latency-bound on its dependent "
                                      "chunk loads and candidate selection, not on HBM or VALU"})
    feats = torch.randn(B, C, N, device=dev)
    g_ms = _time_launches(lambda: K.group_points(feats, idx), 10, stream)
    g_bytes = B * (4 * C * N + 4 * N * Kn + 4 * C * N * Kn)
    roof["grouping_c32"] = roofline_obj("kdpc_group_points", wl, g_ms, 1, g_bytes, 0)
    return roof


# -------------------------------------------------------------------------------- main
def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    sections = set(args.sections.split(","))
    head_mode = args.mode
    head_batch = args.batch
    line = {}
    head = None
    if head_mode in sections:
        head = step_section(args, head_mode, head_batch, dev, world, rank)
    sub_kd = None
    if head_mode == "train" and "kd" in sections:
        sub_kd = step_section(args, "kd", args.kd_batch, dev, world, rank)
    cfg1 = configs1_section(dev) if world == 1 and "configs1" in sections else None
    knn = knn_section(dev) if world == 1 and "knn" in sections else None
    for c in (3, 64):
        if world == 1 and f"gather_c{c}" in sections:
            line[f"gather_c{c}"] = gather_section(dev, c)

    if head is not None:
        line = {
            "metric": "scene-flow pairs/sec fwd+bwd @ N=8192; EPE3D vs ref; 1/2/4/8 MI355X",
            "value": head["value"], "unit": "pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic FlyingThings3D-shaped pairs (kd-pointcloud_amd/synthetic.py), "
                    "random-init weights",
            "config": {"workload": "PointConvBidirection fwd+bwd+Adam (BASELINE configs[2])"
                       if head_mode == "train" else
                       "KD step: teacher fwd + student fwd+bwd + biDirection_loss_ht "
                       "(configs[3])",
                       "model": "models_bid_pointconv.PointConvBidirection",
                       "batch_per_gpu": head_batch, "global_batch": world * head_batch,
                       "npoints": args.npoints, "parallelism": f"dp{world}",
                       "step": head["step"]},
            "host_enqueue_ms": head["host_enqueue_ms"],
            "roofline": head["roofline"],
            "step_roofline": head["step_roofline"],
        }
    if sub_kd is not None:
        sub_kd["workload"] = ("KD step: teacher fwd (eval, no_grad) + student fwd+bwd + "
                              "biDirection_loss_ht(gamma=0.3, beta=0.8, layer=3) + Adam "
                              f"(BASELINE configs[3]: B={args.kd_batch}/GPU, global "
                              f"{world * args.kd_batch})")
        line["kd_step"] = sub_kd
    if cfg1 is not None:
        line["configs1"] = cfg1
        # the north star's gather target, as an HBM figure (inputs rotated past the MALL)
        line["roofline_gather"] = cfg1["grouping_operation_rotated"]
    if knn is not None:
        line["roofline_knn"] = knn
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if head is not None:
            line["cpu_baseline"] = cpu_baseline(args, head_mode)
        if sub_kd is not None:
            sub_kd["cpu_baseline"] = cpu_baseline(args, "kd")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
