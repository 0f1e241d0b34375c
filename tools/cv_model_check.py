"""Record the model's own cost-volume calls (N=2048 trace fixture, student forward) and replay
each D >= 128 call through the fused (kdpc_cost_volume_*) and the unfused wide path on the
same inputs, output by output (diagnostic).

    python tools/cv_model_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import pointconv_util as P
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    calls = []
    orig = P._CostVolume.apply

    def rec(*a):
        if a[3].shape[-1] >= 128:
            # detach, not clone: keep the storages and view offsets the layer saw
            calls.append([t.detach() if torch.is_tensor(t) else t for t in a])
        return orig(*a)
    P._CostVolume.apply = rec
    try:
        T._run_models(g, T._KnnReplay(g))
    finally:
        P._CostVolume.apply = orig
    print(len(calls), "recorded calls")
    import kdpc_native as K
    for ci, a in enumerate(calls):
        x1, x2, idx, p1, p2, wpos, bpos, w1, b1 = a[:9]
        o_f, am_f = K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        h0 = K.cost_volume_wide_h0(x1, x2, idx, p1, p2, wpos, bpos)
        z1 = torch.addmm(b1, h0.view(-1, h0.shape[-1]), w1.t())
        o_u, am_u = K.cost_volume_wide_max(z1, x1.shape[0], x1.shape[1], idx.shape[2], w1.shape[0])
        print(f"call {ci}: amax differs at {int((am_f != am_u).sum())} of {am_f.numel()}, "
              f"max|out diff| {float((o_f - o_u).abs().max()):.3e}")
        res = []
        same = lambda am, _am=am_u: _am  # noqa: E731  (both paths on the unfused routing)
        for fn in (P._CostVolume, P._CostVolumeWide):
            ts = [t.detach().requires_grad_(True) if i not in (2,) and torch.is_tensor(t) else t
                  for i, t in enumerate(a[:9])]
            out = fn.apply(*ts, same)
            torch.manual_seed(5)
            gg = torch.randn_like(out)
            out.backward(gg)
            res.append([out.detach()] + [ts[i].grad for i in (0, 1, 3, 4, 5, 6, 7, 8)])
        names = ["out", "dx1", "dx2", "dp1", "dp2", "dwpos", "dbpos", "dw1", "db1"]
        x1 = a[0]
        print(f"call {ci}: x1 {tuple(x1.shape)} x2 {tuple(a[1].shape)} idx {tuple(a[2].shape)} "
              f"p1 {tuple(a[3].shape)} offsets x1 {x1.storage_offset()} x2 {a[1].storage_offset()} "
              f"idx {a[2].storage_offset()} p1 {a[3].storage_offset()} p2 {a[4].storage_offset()}")
        for nm, u, v in zip(names, res[0], res[1]):
            err = float((u - v).abs().max())
            rel_sum = float((u.double().sum() - v.double().sum()).abs() / (v.double().abs().sum() + 1e-30))
            print(f"  {nm:6s} max|diff| {err:.3e} scale {float(v.abs().max()):.3e} sum-rel {rel_sum:.3e}")


if __name__ == "__main__":
    main()
