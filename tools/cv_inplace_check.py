"""Which inputs of the model's cost-volume calls change between the call and the end of the
backward (N=2048 trace fixture)?  Records every _CostVolume call's inputs both as a clone and
by reference, runs the model's forward + backward, then compares (diagnostic).

    python tools/cv_inplace_check.py
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
    names = ["x1", "x2", "idx", "p1", "p2", "wpos", "bpos", "w1", "b1"]

    def rec(*a):
        calls.append(([t.detach() for t in a[:9]], [t.detach().clone() for t in a[:9]],
                      [t._version for t in a[:9]]))
        return orig(*a)
    P._CostVolume.apply = rec
    try:
        T._run_models(g, T._KnnReplay(g))
    finally:
        P._CostVolume.apply = orig
    torch.cuda.synchronize()
    for ci, (live, snap, ver) in enumerate(calls):
        diffs = [f"{n} (ptr {t.data_ptr():#x}, n={int((t != s).sum())}, version {v}->{t._version})"
                 for n, t, s, v in zip(names, live, snap, ver) if not torch.equal(t, s)]
        print(f"call {ci} p1 {tuple(snap[3].shape)}: " + ("unchanged" if not diffs else
                                                           "CHANGED " + "; ".join(diffs)))


if __name__ == "__main__":
    main()
