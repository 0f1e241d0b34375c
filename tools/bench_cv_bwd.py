"""Cost-volume backward (D <= 64 and the wide widths) at the model's shapes: the ranked entry
point (kdpc_cost_volume_bwd_csr: rows written at their CSR slots, contiguous per-point sums)
vs the plain one (kdpc_cost_volume_bwd: rows in (query, neighbour) order) + CSR gather-sums
through perm (bit-identical dP2 / dx2, checked), on FlyingThings3D-shaped clouds (both
directions of B/2 pairs as one batch of B, as the model runs them).  `--morton` also times the
same calls with the queries renumbered in Morton order of their coordinates (the order the
kernels would walk them in): the per-query arithmetic is unchanged, only the locality of the
gathers and row stores.  HIP events, kernels only (CSR cached).

    python tools/bench_cv_bwd.py [--iters 20] [--morton] [--only cross0]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402
import synthetic  # noqa: E402

DEV = "cuda"
SHAPES = {  # the model's calls at B=8 pairs: both directions as one batch of 16
    "cross0": (16, 8192, 32, 32, 32),
    "cross1": (16, 2048, 32, 64, 64),
    "cross2": (16, 512, 32, 128, 128),
    "cross3": (16, 256, 32, 256, 256),
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


def clouds(B, N, seed=0):
    """Both directions of B/2 FT3D-shaped pairs subsampled to N points: queries, references."""
    p1, p2, _ = synthetic.ft3d_batch(B // 2, 8192, seed=seed)
    rng = np.random.default_rng(seed)
    sel = np.stack([np.sort(rng.choice(8192, N, replace=False)) for _ in range(B // 2)])
    p1 = np.take_along_axis(p1, sel[..., None], 1)
    p2 = np.take_along_axis(p2, sel[..., None], 1)
    q = torch.from_numpy(np.concatenate([p1, p2], 0)).to(DEV).contiguous()
    r = torch.from_numpy(np.concatenate([p2, p1], 0)).to(DEV).contiguous()
    return q, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--morton", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N, Kn, di, do) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        x1, x2 = clouds(B, N)
        p1 = torch.randn(B, N, di, generator=g).to(DEV)
        p2 = torch.randn(B, N, di, generator=g).to(DEV)
        wpos = (torch.randn(di, 3, generator=g) * 0.3).to(DEV)
        bpos = (torch.randn(di, generator=g) * 0.1).to(DEV)
        w1 = (torch.randn(do, di, generator=g) / di ** 0.5).to(DEV)
        b1 = (torch.randn(do, generator=g) * 0.1).to(DEV)
        gout = torch.randn(B, N, do, generator=g).to(DEV)
        variants = [("input", None)]
        if a.morton:
            variants.append(("morton", K._op("kdpc_morton_order", "morton_order", x1).long()))
        for vname, order in variants:
            if order is None:
                q1, qp1, qg = x1, p1, gout
            else:
                perm = lambda t: torch.gather(t, 1, order[..., None].expand(-1, -1, t.shape[-1]))  # noqa: E731
                q1, qp1, qg = perm(x1).contiguous(), perm(p1).contiguous(), perm(gout).contiguous()
            idx = K.knn_point(Kn, x2, q1)
            out, amax = K.cost_volume_fwd(q1, x2, idx, qp1, p2, wpos, bpos, w1, b1)
            csr = K.csr_rank_of(idx, N)  # offsets / perm / rank cached: kernels only below
            res = {}
            if di <= 64:
                def plain():
                    dp1, rows, dx1, drows, dpar = K.cost_volume_bwd(q1, x2, idx, qp1, p2, wpos, bpos,
                                                                    w1, out, amax, qg)
                    dp2 = K.group_rows_grad(rows.view(B, N * Kn, di), csr, B, N, di)
                    dx2 = K.group_rows_grad(drows.view(B, N * Kn, 3), csr, B, N, 3)
                    return dp1, dp2, dx1, dx2, dpar
                r1 = plain()
                res["plain_bwd_plus_sums_us"] = round(timeit(plain, a.iters), 1)
                res["plain_bwd_us"] = round(timeit(lambda: K.cost_volume_bwd(
                    q1, x2, idx, qp1, p2, wpos, bpos, w1, out, amax, qg), a.iters), 1)

            def ranked():
                return K.cost_volume_bwd_csr(q1, x2, idx, qp1, p2, wpos, bpos, w1, out, amax, qg)
            r2 = ranked()
            if di <= 64:
                res["bit_identical"] = all(torch.equal(u, v) for u, v in zip(r1, r2))
            res["fwd_us"] = round(timeit(lambda: K.cost_volume_fwd(q1, x2, idx, qp1, p2, wpos, bpos,
                                                                   w1, b1), a.iters), 1)
            res["ranked_us"] = round(timeit(ranked, a.iters), 1)
            res["checksum_dp2"] = float(r2[1].double().abs().sum())
            print(name, vname, res, flush=True)


if __name__ == "__main__":
    main()
