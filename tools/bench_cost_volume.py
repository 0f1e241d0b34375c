"""Fused cost volume (CrossLayerLight.cross, D <= 64) at the model's shapes: forward and
backward kernel time per call with HIP events on the op's stream.

    python tools/bench_cost_volume.py [--only level0] [--iters 10]

Shapes: cross0 runs on level 0 (N = 8192 per cloud, D 32 -> 32), cross1 on level 1
(N = 2048, D 64 -> 64), K = 32 neighbours; batch = 8 pairs (B = 8 per direction).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
SHAPES = {  # name: (B, N1, N2, K, Din, Dout)
    "level0 (B8 N8192 K32 D32->32)": (8, 8192, 8192, 32, 32, 32),
    "level1 (B8 N2048 K32 D64->64)": (8, 2048, 2048, 32, 64, 64),
}


def timeit(fn, iters, warmup=2):
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
    ap.add_argument("--only", default=None)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N1, N2, Kn, di, do) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        x1 = torch.randn(B, N1, 3, generator=g).to(DEV)
        x2 = torch.randn(B, N2, 3, generator=g).to(DEV)
        idx = K.knn_point(Kn, x2, x1)
        p1 = torch.randn(B, N1, di, generator=g).to(DEV)
        p2 = torch.randn(B, N2, di, generator=g).to(DEV)
        wpos = torch.randn(di, 3, generator=g).to(DEV)
        bpos = torch.randn(di, generator=g).to(DEV)
        w1 = (torch.randn(do, di, generator=g) / di ** 0.5).to(DEV)
        b1 = torch.randn(do, generator=g).to(DEV)
        gout = torch.randn(B, N1, do, generator=g).to(DEV)
        out, amax = K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        f_us = timeit(lambda: K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1), a.iters)
        b_us = timeit(lambda: K.cost_volume_bwd(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax,
                                                gout), a.iters)
        print(name, {"fwd_us": round(f_us, 1), "bwd_us": round(b_us, 1)}, flush=True)


if __name__ == "__main__":
    main()
