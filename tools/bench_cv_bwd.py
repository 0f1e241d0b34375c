"""Cost-volume backward (D <= 64) at the model's shapes: the ranked entry point
(kdpc_cost_volume_bwd_csr: rows written at their CSR slots, contiguous per-point sums) vs the
plain one (kdpc_cost_volume_bwd: rows in (query, neighbour) order) + CSR gather-sums through
perm.  Both give bit-identical dP2 / dx2 (checked).  HIP events, kernels only (CSR cached).

    python tools/bench_cv_bwd.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
SHAPES = {  # the model's two narrow calls at B=8 pairs: both directions as one batch of 16
    "cross0 (B16 N8192 K32 D32)": (16, 8192, 8192, 32, 32, 32),
    "cross1 (B16 N2048 K32 D64)": (16, 2048, 2048, 32, 64, 64),
    "cross2 (B16 N512 K32 D128)": (16, 512, 512, 32, 128, 128),
    "cross3 (B16 N256 K32 D256)": (16, 256, 256, 32, 256, 256),
}


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
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N1, N2, Kn, di, do) in SHAPES.items():
        x1 = torch.rand(B, N1, 3, generator=g).to(DEV)
        x2 = torch.rand(B, N2, 3, generator=g).to(DEV)
        idx = K.knn_point(Kn, x2, x1)
        p1 = torch.randn(B, N1, di, generator=g).to(DEV)
        p2 = torch.randn(B, N2, di, generator=g).to(DEV)
        wpos = torch.randn(di, 3, generator=g).to(DEV)
        bpos = torch.randn(di, generator=g).to(DEV)
        w1 = (torch.randn(do, di, generator=g) / di ** 0.5).to(DEV)
        b1 = torch.randn(do, generator=g).to(DEV)
        gout = torch.randn(B, N1, do, generator=g).to(DEV)
        out, amax = K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        csr = K.csr_rank_of(idx, N2)  # offsets / perm / rank cached: kernels only below

        def plain():
            dp1, rows, dx1, drows, dpar = K.cost_volume_bwd(x1, x2, idx, p1, p2, wpos, bpos, w1,
                                                            out, amax, gout)
            dp2 = K.group_rows_grad(rows.view(B, N1 * Kn, di), csr, B, N2, di)
            dx2 = K.group_rows_grad(drows.view(B, N1 * Kn, 3), csr, B, N2, 3)
            return dp1, dp2, dx1, dx2, dpar

        def ranked():
            return K.cost_volume_bwd_csr(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout)
        r1, r2 = plain(), ranked()
        same = all(torch.equal(u, v) for u, v in zip(r1, r2))
        t_plain = timeit(plain, a.iters)
        t_bwd = timeit(lambda: K.cost_volume_bwd(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax,
                                                 gout), a.iters)
        t_ranked = timeit(ranked, a.iters)
        res = {"plain_bwd_plus_sums_us": round(t_plain, 1), "plain_bwd_us": round(t_bwd, 1),
               "ranked_us": round(t_ranked, 1), "bit_identical": same}
        print(name, res, flush=True)


if __name__ == "__main__":
    main()
