"""Fused PointConv layer at the model's shapes (batch 8 pairs, N=8192): forward and backward
time per call with HIP events (and the weight half alone, as the side stream runs it), and
the f32 MFMA rate they reach.

    python tools/bench_pointconv.py [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
# name: (B, N, S, K, D, O) -- encoder levels run on the pair batch (2B = 16)
SHAPES = {
    "flow0_pc1 (B8 N8192 K9 D128 O128)": (8, 8192, 8192, 9, 128, 128),
    "flow1_pc1 (B8 N2048 K9 D192 O128)": (8, 2048, 2048, 9, 192, 128),
    "level1 (2B16 N8192 S2048 K16 D64 O64)": (16, 8192, 2048, 16, 64, 64),
    "level3 (2B16 N512 S256 K16 D256 O256)": (16, 512, 256, 16, 256, 256),
    "level4 (2B16 N256 S64 K16 D512 O256)": (16, 256, 64, 16, 512, 256),
}


def timeit(fn, iters=10, warmup=2):
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


def morton_sort(xyz, bits=10):
    lo = xyz.amin(1, keepdim=True)
    hi = xyz.amax(1, keepdim=True)
    q = ((xyz - lo) / (hi - lo + 1e-9) * (2 ** bits - 1)).long()
    code = torch.zeros(xyz.shape[:2], dtype=torch.long, device=xyz.device)
    for b in range(bits):
        for a in range(3):
            code |= ((q[..., a] >> b) & 1) << (3 * b + a)
    order = code.argsort(1)
    return torch.gather(xyz, 1, order.unsqueeze(-1).expand(-1, -1, 3)).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="substring of the shape names to run")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dump", default=None, help="save every backward output here (.npz)")
    ap.add_argument("--morton", action="store_true",
                    help="sort each cloud by a Morton code first (spatially coherent rows)")
    args = ap.parse_args()
    res = {}
    dump = {}
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N, S, Kn, D, O) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        xyz = torch.randn(B, N, 3, generator=g).to(DEV)
        if args.morton:
            xyz = morton_sort(xyz)
        center = xyz[:, :S].contiguous()
        feats = torch.randn(B, N, D, generator=g).to(DEV)
        idx = K.knn_point(Kn, xyz, center)
        wt = torch.randn(B, S, Kn, 16, generator=g).to(DEV)
        C = 3 + D
        wl = (torch.randn(O, 16 * C, generator=g) / (16 * C) ** 0.5).to(DEV)
        bias = torch.randn(O, generator=g).to(DEV)
        dy = torch.randn(B, S, O, generator=g).to(DEV)
        csr = K.csr_of(idx, N)
        fwd = timeit(lambda: K.pointconv_fwd(xyz, center, feats, idx, wt, wl, bias), args.iters)
        bwd = timeit(lambda: K.pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, csr,
                                             need_xyz=False), args.iters)
        wgt = timeit(lambda: K.pointconv_bwd_weight(xyz, center, feats, idx, wt, dy, O),
                     args.iters)
        if args.dump:
            dump[f"{name}/dwl"] = K.pointconv_bwd_weight(xyz, center, feats, idx, wt, dy,
                                                         O).cpu().numpy()
            outs = K.pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=True)
            for i, o in enumerate(outs):
                if torch.is_tensor(o):
                    dump[f"{name}/{i}"] = o.cpu().numpy()
        R = B * S
        gemm = 2.0 * R * 16 * C * O
        build = 2.0 * R * Kn * C * 16
        res[name] = {"fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1), "weight_us": round(wgt, 1),
                     "weight_TFLOPs": round((gemm + build) / (wgt * 1e-6) / 1e12, 1),
                     "fwd_TFLOPs": round((gemm + build) / (fwd * 1e-6) / 1e12, 1),
                     "bwd_TFLOPs": round((2 * gemm + 3 * build) / (bwd * 1e-6) / 1e12, 1)}
        print(name, res[name], flush=True)
    if args.dump:
        import numpy as np
        np.savez(args.dump, **dump)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
