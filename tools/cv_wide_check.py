"""Compare the fused wide cost volume (kdpc_cost_volume_fwd/_bwd at D = 128/256) with the
unfused wide path (cvw_* kernels + BLAS) on identical inputs, output by output (diagnostic).

    python tools/cv_wide_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))

import torch  # noqa: E402


def main():
    import pointconv_util as P
    import synthetic
    dev = "cuda"
    for (d, n1, n2, b, k) in [(128, 128, 128, 2, 32), (128, 128, 128, 1, 32), (256, 64, 64, 2, 32),
                              (128, 300, 280, 2, 32)]:
        torch.manual_seed(d + n1 + b)
        x1 = torch.from_numpy(synthetic.ft3d_batch(b, n1, seed=1)[0]).to(dev)
        x2 = torch.from_numpy(synthetic.ft3d_batch(b, n2, seed=2)[0]).to(dev)
        p1 = torch.randn(b, n1, d, device=dev)
        p2 = torch.randn(b, n2, d, device=dev)
        wpos = torch.randn(d, 3, device=dev) * 0.3
        bpos = torch.randn(d, device=dev) * 0.1
        w1 = torch.randn(d, d, device=dev) / d ** 0.5
        b1 = torch.randn(d, device=dev) * 0.1
        idx = P.knn_point(k, x2, x1)
        idx = P._as_idx32(idx).contiguous()
        res = []
        for fn in (P._CostVolume, P._CostVolumeWide):
            ts = [t.detach().clone().requires_grad_(True) for t in (x1, x2, p1, p2, wpos, bpos, w1, b1)]
            a1, a2, q1, q2, wp, bp, ww, bb = ts
            out = fn.apply(a1, a2, idx, q1, q2, wp, bp, ww, bb, None)
            torch.manual_seed(5)
            g = torch.randn_like(out)
            out.backward(g)
            res.append([out.detach()] + [t.grad for t in ts])
        names = ["out", "dx1", "dx2", "dp1", "dp2", "dwpos", "dbpos", "dw1", "db1"]
        print(f"D={d} n1={n1} n2={n2} B={b} K={k}")
        for nm, a, c in zip(names, res[0], res[1]):
            err = float((a - c).abs().max())
            scale = float(c.abs().max())
            rel_sum = float((a.double().sum() - c.double().sum()).abs() / c.double().abs().sum())
            print(f"  {nm:6s} max|diff| {err:.3e}  scale {scale:.3e}  sum-rel {rel_sum:.3e}")


if __name__ == "__main__":
    main()
