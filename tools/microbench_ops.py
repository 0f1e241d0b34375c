"""Per-op microbenchmarks (BASELINE configs[1] and configs[4]) with HIP-event timing.

    python tools/microbench_ops.py [--json out.json]

config 2: B=8, N=8192: FPS 8192->2048, ball_query r=0.5 K=16 (S=2048), grouping C=64 S=2048
          K=16 (fwd + deterministic bwd), gather of xyz; plus a cache-busting grouping
          variant (B=32, S=N=8192) whose working set exceeds the 256 MiB Infinity Cache.
config 5: kNN K=32, N=65536 refs / 65536 queries per frame, B=4.
Algorithmic bytes follow SURVEY §8d.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402
import synthetic  # noqa: E402

DEV = "cuda"


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
    return s.elapsed_time(e) / iters * 1e3  # us


def cloud(b, n, seed):
    p1, _, _ = synthetic.ft3d_batch(b, n, seed=seed)
    return torch.from_numpy(p1).to(DEV)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    res = {}
    B, N, S, Kn, C = 8, 8192, 2048, 16, 64
    xyz = cloud(B, N, 1)
    # FPS
    us = timeit(lambda: K.furthest_point_sampling(xyz, S), iters=5, warmup=1)
    res["fps_8192_to_2048_B8"] = {"us": us, "us_per_step": us / (S - 1),
                                  "dist_updates_per_s": B * N * (S - 1) / (us * 1e-6)}
    idx_fps = K.furthest_point_sampling(xyz, S)
    new_xyz = K.group_rows(xyz, idx_fps)
    # ball query
    us = timeit(lambda: K.ball_query(0.5, Kn, xyz, new_xyz))
    res["ball_query_r0.5_K16_B8"] = {"us": us}
    # grouping (B,C,N) API, C=64
    feats = torch.randn(B, C, N, device=DEV)
    idx = K.ball_query(0.5, Kn, xyz, new_xyz)
    nbytes = B * (4 * C * N + 4 * S * Kn + 4 * C * S * Kn)
    us = timeit(lambda: K.group_points(feats, idx))
    res["group_points_fwd_C64_S2048_K16_B8"] = {"us": us, "GBps": nbytes / (us * 1e-6) / 1e9,
                                                "algorithmic_bytes": nbytes}
    gout = torch.randn(B, C, S, Kn, device=DEV)
    csr = K.csr_of(idx, N)
    us = timeit(lambda: K.csr_sum_channels(gout, csr, B, C, N))
    res["group_points_bwd_C64_S2048_K16_B8"] = {"us": us, "GBps": nbytes / (us * 1e-6) / 1e9}
    us = timeit(lambda: K.Csr(idx.view(B, -1), N))
    res["csr_build_B8_P32768"] = {"us": us}
    # point-major rows (what the layers use)
    rows = feats.transpose(1, 2).contiguous()
    rbytes = B * (4 * S * Kn + 8 * S * Kn * C)
    us = timeit(lambda: K.group_rows(rows, idx.view(B, -1)))
    res["group_rows_fwd_C64_S2048_K16_B8"] = {"us": us, "GBps": rbytes / (us * 1e-6) / 1e9}
    # gather of xyz (B,3,N) -> (B,3,S)
    xyz_cn = xyz.transpose(1, 2).contiguous()
    us = timeit(lambda: K.gather_points(xyz_cn, idx_fps))
    res["gather_points_xyz_B8"] = {"us": us}
    # cache-busting grouping: B=32, S=N=8192, K=16, C=64 (out = 1 GiB)
    Bb = 32
    xb = cloud(Bb, N, 2)
    ib = K.knn_point(Kn, xb, xb)
    fb = torch.randn(Bb, C, N, device=DEV)
    nb = Bb * (4 * C * N + 4 * N * Kn + 4 * C * N * Kn)
    us = timeit(lambda: K.group_points(fb, ib), iters=5)
    res["group_points_fwd_cachebust_B32_S8192"] = {"us": us, "GBps": nb / (us * 1e-6) / 1e9}
    del fb
    # kNN config 5
    x5 = cloud(4, 65536, 3)
    q5 = cloud(4, 65536, 4)
    us = timeit(lambda: K.knn_point(32, x5, q5), iters=2, warmup=1)
    res["knn_K32_N65536_B4"] = {"us": us, "Gdist_per_s": 4 * 65536 * 65536 / (us * 1e-6) / 1e9,
                                "algorithmic_bytes": 4 * (12 * 65536 * 2 + 4 * 65536 * 32)}
    us = timeit(lambda: K.knn_point(32, x5, q5, seeded=False), iters=2, warmup=1)
    res["knn_K32_N65536_B4_plain"] = {"us": us}
    us = timeit(lambda: K.knn_point(32, xyz, xyz), iters=5)
    res["knn_K32_self_N8192_B8"] = {"us": us, "Gdist_per_s": B * N * N / (us * 1e-6) / 1e9}
    # the model's kNN shapes, seeded vs unseeded scan
    x16 = cloud(16, N, 5)
    for (b, n, s, k) in [(16, 8192, 8192, 32), (8, 8192, 8192, 9), (16, 2048, 2048, 32),
                         (8, 2048, 2048, 9), (16, 512, 512, 32), (8, 8192, 2048, 3)]:
        xr, xq = x16[:b, :n].contiguous(), x16[:b, :s].flip(1).contiguous()
        for seeded in (True, False):
            us = timeit(lambda: K.knn_point(k, xr, xq, seeded=seeded), iters=10)
            res[f"knn_B{b}_N{n}_S{s}_K{k}_{'seeded' if seeded else 'plain'}"] = {"us": us}
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
