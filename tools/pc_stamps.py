"""Diagnostic (GPU): where the PointConv backward data kernel spends a chunk.

Needs the KDPC_DAT_MODE=9 build (per-wave s_memtime stamps of every chunk phase, copied to
a device buffer of their own):

    bash tools/build_variants.sh stamps:-DKDPC_DAT_MODE=9
    KDPC_LIB=tools/variants/stamps/libkdpc_hip.so python tools/pc_stamps.py [--json out]

Per chunk and wave, the phases between stamps:
  mfma   chunk top -> after the dA MFMAs, the next chunk's B / gather loads issued
  sync1  -> dA stored to LDS (waits for the MFMA results) + barrier
  valu   -> the pair phase (dG / dwt fmas, dG stores issued)
  sync2  -> barrier + the next chunk's gathers landed (next chunk top)
Read the shares, not the absolute time: the stamps' waits forbid overlaps the real kernel has.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

NWG, NS = 4096, 80


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--shape", default="8,8192,8192,9,128,128", help="B,N,S,K,D,O")
    ap.add_argument("--morton", action="store_true")
    ap.add_argument("--weight", action="store_true",
                    help="the weight kernel's phase sums (KDPC_WGT_MODE=9 build)")
    args = ap.parse_args()
    B, N, S, Kn, D, O = (int(x) for x in args.shape.split(","))
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    xyz = torch.randn(B, N, 3, generator=g).to(dev)
    if args.morton:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_pointconv import morton_sort
        xyz = morton_sort(xyz)
    center = xyz[:, :S].contiguous()
    feats = torch.randn(B, N, D, generator=g).to(dev)
    idx = K.knn_point(Kn, xyz, center)
    wt = torch.randn(B, S, Kn, 16, generator=g).to(dev)
    C = 3 + D
    wl = (torch.randn(O, 16 * C, generator=g) / (16 * C) ** 0.5).to(dev)
    dy = torch.randn(B, S, O, generator=g).to(dev)
    csr = K.csr_of(idx, N)
    for _ in range(5):
        K.pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=False)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["KDPC_LIB"])
    if args.weight:
        buf = np.zeros(4096 * 8 * 8, dtype=np.uint64)
        rc = lib.kdpc_debug_pcw_stamps(buf.ctypes.data_as(ctypes.c_void_p),
                                       ctypes.c_size_t(buf.nbytes))
        assert rc == 0, rc
        st = buf.reshape(4096, 8, 8).astype(np.int64)
        st = st[st[:, 0, 7] > 0]  # workgroups that ran tiles
        names = ["prologue", "fetch_issue", "mfma_issue", "build", "sync1", "stage", "sync2"]
        tot = st[:, :, :7].sum(-1)
        res = {"shape": args.shape, "workgroups": int(st.shape[0]),
               "tiles_per_wg": float(st[:, 0, 7].mean()),
               "wave_cycles_mean": float(tot.mean()),
               "cycles_per_tile": float((tot - st[:, :, 0]).mean() / st[:, 0, 7].mean()),
               "share": {n: float((st[:, :, i] / tot).mean()) for i, n in enumerate(names)},
               "share_by_wave": {n: [round(float((st[:, w, i] / tot[:, w]).mean()), 3)
                                     for w in range(8)] for i, n in enumerate(names)}}
        print(json.dumps(res, indent=1))
        if args.json:
            json.dump(res, open(args.json, "w"), indent=1)
        return
    buf = np.zeros(NWG * 4 * NS, dtype=np.uint64)
    rc = lib.kdpc_debug_pc_stamps(buf.ctypes.data_as(ctypes.c_void_p),
                                  ctypes.c_size_t(buf.nbytes))
    assert rc == 0, rc
    nwg = min(NWG, (B * S + 31) // 32)
    st = buf.reshape(NWG, 4, NS)[:nwg].astype(np.int64)
    nch = (C + 7) // 8
    t0 = st[:, :, 0]
    tend = st[:, :, 78]
    res = {"shape": args.shape, "workgroups": nwg, "chunks": nch}
    total = tend - t0
    res["wave_cycles_mean"] = float(total.mean())
    res["prologue_share"] = float(((st[:, :, 1] - t0) / total).mean())
    phases = {"mfma": [], "sync1": [], "valu": [], "sync2": []}
    for i in range(nch):
        a, b, c, d = (st[:, :, 2 + 4 * i + j] for j in range(4))
        nxt = st[:, :, 2 + 4 * (i + 1)] if i + 1 < nch else tend
        for name, v in zip(phases, (b - a, c - b, d - c, nxt - d)):
            phases[name].append(v)
    per = {k: np.stack(v, -1) for k, v in phases.items()}  # (wg, wave, chunk)
    chunk_total = sum(per.values())
    res["chunk_cycles_mean"] = float(chunk_total.mean())
    res["phase_cycles_mean"] = {k: float(v.mean()) for k, v in per.items()}
    res["phase_cycles_by_wave"] = {k: [float(v[:, w].mean()) for w in range(4)]
                                   for k, v in per.items()}
    res["phase_cycles_chunk0_vs_rest"] = {k: [float(v[:, :, 0].mean()), float(v[:, :, 1:].mean())]
                                          for k, v in per.items()}
    # workgroup schedule: start offsets (rounds) and per-XCC counts
    start = t0[:, 0] - t0[:, 0].min()
    res["wg_start_quantiles_cycles"] = [float(np.quantile(start, q)) for q in (0, .25, .5, .75, 1)]
    res["wg_cycles_quantiles"] = [float(np.quantile(total[:, 0], q)) for q in (0, .1, .5, .9, 1)]
    xcc = (st[:, 0, 79] >> 32) & 0xF
    res["wg_per_xcc"] = np.bincount(xcc, minlength=8).tolist()
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
