"""Wide cost volume (D in {128, 256}, one-kernel MFMA path) at the model's cross2 / cross3
calls (B=16 pair batch, K=32): forward and backward (with the CSR sums) per call, HIP events.

    python tools/bench_cv_wide.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
SHAPES = {"cross2 (B16 N512 K32 D128)": (16, 512, 32, 128),
          "cross3 (B16 N256 K32 D256)": (16, 256, 32, 256)}


def timeit(fn, iters=20, warmup=3):
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
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N, Kn, D) in SHAPES.items():
        x1 = torch.rand(B, N, 3, generator=g).to(DEV)
        x2 = torch.rand(B, N, 3, generator=g).to(DEV)
        idx = K.knn_point(Kn, x2, x1)
        p1 = torch.randn(B, N, D, generator=g).to(DEV)
        p2 = torch.randn(B, N, D, generator=g).to(DEV)
        wpos = torch.randn(D, 3, generator=g).to(DEV)
        bpos = torch.randn(D, generator=g).to(DEV)
        w1 = (torch.randn(D, D, generator=g) / D ** 0.5).to(DEV)
        b1 = torch.randn(D, generator=g).to(DEV)
        gout = torch.randn(B, N, D, generator=g).to(DEV)
        out, amax = K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        t_f = timeit(lambda: K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1))
        t_b = timeit(lambda: K.cost_volume_bwd_csr(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax,
                                                   gout))
        print(name, {"fwd_us": round(t_f, 1),
              "bwd_csr_us": round(t_b, 1), "checksum": float(out.double().sum())}, flush=True)


if __name__ == "__main__":
    main()
