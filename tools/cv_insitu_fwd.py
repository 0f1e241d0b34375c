"""In-situ check of the fused cost-volume FORWARD inside the model run (N=2048 trace
fixture): every call's out / amax vs a float64 torch evaluation of the same inputs
(diagnostic).

    python tools/cv_insitu_fwd.py
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
    import kdpc_native as K
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    orig = K.cost_volume_fwd
    seen = []

    def wrapped(x1, x2, idx, p1, p2, wpos, bpos, w1, b1):
        out, am = orig(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        torch.cuda.synchronize()
        d = lambda t: t.detach().double()  # noqa: E731
        B, N1, Kk = idx.shape
        bi = torch.arange(B, device=idx.device).view(B, 1, 1)
        il = idx.long()
        dirn = d(x2)[bi, il] - d(x1).unsqueeze(2)
        h0 = torch.nn.functional.leaky_relu(d(p2)[bi, il] + d(p1).unsqueeze(2)
                                            + dirn @ d(wpos).t() + d(bpos), 0.1)
        z = torch.nn.functional.leaky_relu(h0 @ d(w1).t() + d(b1), 0.1)
        ref = z.max(2)[0]
        err = (out.double() - ref).abs()
        # routing: z at the build's argmax must be within rounding of the max
        zsel = torch.gather(z, 2, am.long().unsqueeze(2)).squeeze(2)
        gap = (ref - zsel).abs()
        seen.append((tuple(p1.shape), float(err.max()), float(ref.abs().max()),
                     int((gap > 1e-4 * ref.abs().max()).sum()), float(gap.max())))
        return out, am
    K.cost_volume_fwd = wrapped
    try:
        T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    finally:
        K.cost_volume_fwd = orig
    for s in seen:
        print("p1 %s: out max|err| %.2e (scale %.2e); wrong-routing entries %d (max gap %.2e)" % s,
              flush=True)


if __name__ == "__main__":
    main()
