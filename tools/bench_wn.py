"""WeightNet backward alone (kdpc_weightnet_bwd: parameter half, and the drel half) at the
train step's shapes, HIP events, kernel-only timing per call.

    python tools/bench_wn.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
# (B, N refs, S rows' centers, K): flow estimators at levels 0-3 (B=8), encoder levels (pair
# batch 16)
SHAPES = [(8, 8192, 8192, 9), (8, 2048, 2048, 9), (16, 8192, 2048, 16), (16, 2048, 512, 16),
          (16, 512, 256, 16)]


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    params = [torch.randn(8, 3, generator=g), torch.randn(8, generator=g),
              torch.randn(8, 8, generator=g), torch.randn(8, generator=g),
              torch.randn(16, 8, generator=g), torch.randn(16, generator=g)]
    params = [p.to(DEV) * 0.5 for p in params]
    for b, n, s, k in SHAPES:
        xyz = torch.rand(b, n, 3, generator=g).to(DEV)
        center = torch.rand(b, s, 3, generator=g).to(DEV)
        idx = torch.randint(0, n, (b, s, k), generator=g, dtype=torch.int32).to(DEV)
        dwt = torch.randn(b, s, k, 16, generator=g).to(DEV)
        t_par = timeit(lambda: K.weightnet_bwd(xyz, center, idx, params, dwt, False))
        t_rel = timeit(lambda: K.weightnet_bwd_rel(xyz, center, idx, params, dwt))
        _, dp = K.weightnet_bwd(xyz, center, idx, params, dwt, False)
        print(f"B={b} N={n} S={s} K={k} rows={b * s * k}: params half {t_par:.1f} us, drel half "
              f"{t_rel:.1f} us, |dparams| checksum {float(dp.abs().sum()):.6e}", flush=True)


if __name__ == "__main__":
    main()
