"""What-if step timing: the graphed training step (bench configs[2]: B=8, N=8192) with one
piece of work replaced by an allocation of the right shape, to bound what optimising that
piece could gain.  Diagnostic only (the gradients it produces are wrong); every variant runs
in its own child process.

    python tools/whatif.py [--variants base,no_wn_param,...] [--steps 20]

Variants: base; no_wn_param (WeightNet parameter reduction); no_pc_weight (PointConv weight
kernel); no_pc_data (PointConv data kernel + CSR sums); no_cv_bwd (every cost-volume backward);
no_cv_narrow_bwd (the D <= 64 ones); no_colsum (every fixed-order column sum issued from
Python); no_splitk (dense split-K weight GEMMs); no_side (the four parameter-gradient pieces
together).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kd-pointcloud_amd")


def patch(variant):
    if variant == "no_side":  # every parameter-gradient stream launch
        for v in ("no_wn_param", "no_pc_weight", "no_colsum", "no_splitk"):
            patch(v)
        return
    import torch
    import kdpc_native as K
    import dense

    if variant == "no_wn_param":
        def wb(xyz, center, idx, params, dwt, need_rel=False):
            n = sum(p.numel() for p in params)
            return None, torch.zeros(n, device=xyz.device)
        K.weightnet_bwd = wb
    elif variant == "no_pc_weight":
        def w(xyz, center, feats, idx, wt, dy, o):
            return torch.zeros(o, 16 * (3 + feats.shape[2]), device=xyz.device)

        def wbias(xyz, center, feats, idx, wt, dy, o):
            return w(xyz, center, feats, idx, wt, dy, o), torch.zeros(o, device=xyz.device)
        K.pointconv_bwd_weight, K.pointconv_bwd_weight_bias = w, wbias
    elif variant == "no_pc_data":
        def z(xyz, feats, idx, need_xyz):
            B, N, _ = xyz.shape
            S, Kk = idx.shape[1], idx.shape[2]
            t = lambda *s: torch.zeros(*s, device=xyz.device)  # noqa: E731
            return (t(B, N, 3) if need_xyz else None, t(B, N, feats.shape[2]), t(B, S, 3),
                    t(B, S, Kk, 16))
        K.pointconv_bwd_data = lambda xyz, center, feats, idx, wt, wl, dy, csr, need_xyz=True: \
            z(xyz, feats, idx, need_xyz)
        K.pointconv_bwd_tiled = lambda xyz, center, feats, idx, wt, wl, dy, tp, need_xyz=True, \
            weight=True: z(xyz, feats, idx, need_xyz) + (None,)
    elif variant in ("no_cv_bwd", "no_cv_narrow_bwd"):
        orig = K.cost_volume_bwd_csr

        def cvb(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout, slope0=None):
            din, dout = p1.shape[2], w1.shape[0]
            if variant == "no_cv_narrow_bwd" and din > 64:
                return orig(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout, slope0)
            z = lambda *s: torch.zeros(*s, device=x1.device)  # noqa: E731
            return (z(*p1.shape), z(*p2.shape), z(*x1.shape), z(*x2.shape),
                    z(dout * din + dout + 4 * din))
        K.cost_volume_bwd_csr = cvb
    elif variant == "no_colsum":
        K.colsum = lambda x2: torch.zeros(x2.shape[-1], device=x2.device)
    elif variant == "no_splitk":
        dense.splitk_tn = lambda a, b: torch.zeros(a.shape[-1], b.shape[-1], device=a.device)
    elif variant != "base":
        raise SystemExit(f"unknown variant {variant}")


def child(variant, steps, warmup):
    sys.path.insert(0, PKG)
    import torch
    import synthetic
    from distill import graphed_flow_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    patch(variant)
    dev = torch.device("cuda", 0)
    batches = []
    for i in range(4):
        p1, p2, fl = synthetic.ft3d_batch(8, 8192, seed=1000, first_pair=i * 8)
        batches.append(tuple(torch.from_numpy(a).to(dev) for a in (p1, p2, fl)))
    torch.manual_seed(0)
    model = PointConvBidirection().to(dev)
    opt = make_optimizer(model, capturable=True)
    step = graphed_flow_step(model, opt, batches[0])
    nxt = lambda i: {"next_batch": batches[(i + 1) % 4]}  # noqa: E731
    for i in range(warmup):
        step(*batches[i % 4], **nxt(i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(*batches[i % 4], **nxt(i))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({"variant": variant, "ms_per_step": round(ms, 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,no_wn_param,no_pc_weight,no_pc_data,no_cv_bwd,"
                    "no_cv_narrow_bwd,no_colsum,no_splitk,no_side")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.steps, a.warmup)
        return
    for v in a.variants.split(",") * a.rounds:
        r = subprocess.run([sys.executable, __file__, "--child", v, "--steps", str(a.steps),
                            "--warmup", str(a.warmup)], capture_output=True, text=True,
                           timeout=400)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        print(line[-1] if line else f"{v}: failed rc={r.returncode} {r.stderr[-800:]}",
              flush=True)


if __name__ == "__main__":
    main()
