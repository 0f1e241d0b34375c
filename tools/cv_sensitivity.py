"""Is the cross1 divergence between the fused-wide and unfused-wide model runs a LeakyReLU'
sign flip at a near-zero pre-activation (a tie of the math, like a kNN or max near-tie)?
Records the D=64 cost-volume inputs of both runs and evaluates each in float64 with the same
incoming gradient (diagnostic).

    python tools/cv_sensitivity.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import cv_localise as L  # noqa: E402


def pre_act(x1, x2, idx, p1, p2, wpos, bpos):
    d = lambda t: t.detach().double()  # noqa: E731
    B = idx.shape[0]
    bi = torch.arange(B, device=idx.device).view(B, 1, 1)
    il = idx.long()
    dirn = d(x2)[bi, il] - d(x1).unsqueeze(2)
    return d(p2)[bi, il] + d(p1).unsqueeze(2) + dirn @ d(wpos).t() + d(bpos)


def run(narrow_only):
    import kdpc_native as K
    import pointconv_util as P
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    sup = K.cost_volume_supported
    if narrow_only:
        K.cost_volume_supported = lambda din, dout, k: din in (32, 64) and dout in (32, 64)
    calls = []
    orig = P._CostVolume.apply

    def rec(*a):
        out = orig(*a)
        if torch.is_grad_enabled():
            calls.append([t.detach().clone() for t in a[:9]] + [out.detach().clone(),
                                                                 amaxes[-1]])
        return out
    P._CostVolume.apply = rec
    amaxes = []
    rep = T._AmaxReplay(g64)

    def amax_rec(am):
        r = rep(am)
        amaxes.append(r.clone())
        return r
    try:
        T._run_models(g, T._KnnReplay(g), amax_rec)
    finally:
        P._CostVolume.apply = orig
        K.cost_volume_supported = sup
    return calls


def main():
    ca = run(False)
    cb = run(True)
    # the student's narrow calls (D <= 64) are recorded in both runs in the same order
    na = [(c, c[10]) for c in ca if c[3].shape[-1] <= 64]
    nb = [(c, c[10]) for c in cb if c[3].shape[-1] <= 64]
    for (c1, a1), (c2, a2) in zip(na, nb):
        h1, h2 = pre_act(*c1[:7]), pre_act(*c2[:7])
        flips = int(((h1 > 0) != (h2 > 0)).sum())
        torch.manual_seed(3)
        gout = torch.randn_like(c1[9])
        r1 = L.f64_grads(*c1[:9], a1, gout)
        r2 = L.f64_grads(*c2[:9], a2, gout)
        rel = lambda u, v: float((u - v).abs().max()) / float(v.abs().max())  # noqa: E731
        print(f"p1 {tuple(c1[3].shape)}: inputs rel {rel(c1[3].double(), c2[3].double()):.1e}; "
              f"pre-activation sign flips {flips} (min |pre| {float(h1.abs().min()):.1e}); "
              f"float64 dp1 rel {rel(r1[0], r2[0]):.2e} dp2 rel {rel(r1[6], r2[6]):.2e} "
              f"dW1 rel {rel(r1[2], r2[2]):.2e}", flush=True)


if __name__ == "__main__":
    main()
