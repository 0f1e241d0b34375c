"""PointConv backward data half at the estimators' shapes (B=8 pairs, synthetic
FlyingThings-shaped clouds, self-kNN K=9): untiled (one dG row per pair + kNN CSR sum) vs
tiled (dG summed per Morton-ordered 32-row tile and destination in the kernel).  HIP events,
kernels only (plans built once, outside the timing).

    python tools/bench_pc_tiled.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402
import pointconv_util as P  # noqa: E402
import synthetic  # noqa: E402

DEV = "cuda"
SHAPES = {"flow0 (N8192 D128)": (8192, 128), "flow1 (N2048 D192)": (2048, 192),
          "flow2 (N512 D320)": (512, 320)}


def timeit(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    p1, _, _ = synthetic.ft3d_batch(8, 8192, seed=3)
    full = torch.from_numpy(p1).to(DEV)
    if full.shape[1] == 3:
        full = full.transpose(1, 2).contiguous()
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (n, d) in SHAPES.items():
        xyz = full[:, :n].contiguous()
        b, o, k = xyz.shape[0], 128, 9
        idx = P._as_idx32(P.knn_point(k, xyz, xyz)).contiguous()
        feats = torch.randn(b, n, d, generator=g).to(DEV)
        wt = torch.randn(b, n, k, 16, generator=g).to(DEV)
        wl = (torch.randn(o, 16 * (3 + d), generator=g) * 0.05).to(DEV)
        dy = torch.randn(b, n, o, generator=g).to(DEV)
        csr = K.csr_rank_of(idx, n)
        tp = K.tile_plan_of(idx, xyz, n)
        nrows = int(tp.offsets[-1])
        t_u = timeit(lambda: K.pointconv_bwd_data(xyz, xyz, feats, idx, wt, wl, dy, csr),
                     a.iters)
        t_t = timeit(lambda: K.pointconv_bwd_tiled(xyz, xyz, feats, idx, wt, wl, dy, tp,
                                                   weight=False), a.iters)
        bias = torch.randn(o, generator=g).to(DEV)
        f_u = timeit(lambda: K.pointconv_fwd(xyz, xyz, feats, idx, wt, wl, bias), a.iters)
        f_t = timeit(lambda: K.pointconv_fwd_tiled(xyz, xyz, feats, idx, wt, wl, bias, tp.trow),
                     a.iters)
        print(name, {"fwd_untiled_us": round(f_u, 1), "fwd_tiled_us": round(f_t, 1)},
              flush=True)
        print(name, {"untiled_us": round(t_u, 1), "tiled_us": round(t_t, 1),
                     "dG_rows_untiled": b * n * k, "dG_rows_tiled": nrows}, flush=True)


if __name__ == "__main__":
    main()
