"""In-situ check of the fused wide cost-volume backward inside the model run (N=2048 trace
fixture, float64 max routing replayed): every D >= 128 backward call is also evaluated in
float64 torch on the very tensors the fused backward received (diagnostic).

    python tools/cv_insitu.py
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


def main():
    import kdpc_native as K
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    import pointconv_util as P
    orig = K.cost_volume_bwd_csr
    seen = []
    b1_of = {}
    orig_apply = P._CostVolume.apply

    def rec(*a):
        b1_of[a[7].data_ptr()] = a[8].detach()
        return orig_apply(*a)
    P._CostVolume.apply = rec

    def wrapped(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout):
        res = orig(x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, gout)
        D = w1.shape[0]
        if D >= 128:
            torch.cuda.synchronize()
            b1 = b1_of[w1.data_ptr()]
            with torch.enable_grad():
                ref = L.f64_grads(x1, x2, idx, p1, p2, wpos, bpos, w1, b1, amax, gout)
            dp1, dp2, dx1, dx2, dpar = res
            e = lambda a, b: float((a.double() - b).abs().max()) / (float(b.abs().max()) + 1e-30)  # noqa
            db1 = dpar[D * D:D * D + D]
            din = p1.shape[-1]
            dwpos = dpar[D * D + D:D * D + D + 3 * din].view(3, din).t()
            dbpos = dpar[D * D + D + 3 * din:]
            seen.append((tuple(p1.shape), e(dp1, ref[0]), e(dx1, ref[1]),
                         e(dpar[:D * D].view(D, D), ref[2]), e(db1, ref[3]),
                         e(dwpos, ref[4]), e(dbpos, ref[5]), e(dp2, ref[6]), e(dx2, ref[7]),
                         float(gout.abs().max()), int((gout == 0).sum()), gout.is_contiguous(),
                         int(amax.max()), out.is_contiguous()))
        return res
    K.cost_volume_bwd_csr = wrapped
    try:
        T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    finally:
        K.cost_volume_bwd_csr = orig
        P._CostVolume.apply = orig_apply
    for s in seen:
        print("p1 %s: rel err dp1 %.2e dx1 %.2e dW1 %.2e db1 %.2e dWpos %.2e dbpos %.2e dp2 %.2e "
              "dx2 %.2e | |gout| %.2e zeros %d contig %s "
              "amax max %d out contig %s" % s, flush=True)


if __name__ == "__main__":
    main()
