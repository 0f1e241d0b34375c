"""Fused vs unfused wide cost volume: the student's parameter gradients of two full model runs
(N=2048 trace fixture, float64 routing replayed), element by element (diagnostic).

    python tools/grad_runs_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def grads(narrow_only):
    import kdpc_native as K
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    sup = K.cost_volume_supported
    if narrow_only:
        K.cost_volume_supported = lambda din, dout, k: din in (32, 64) and dout in (32, 64)
    try:
        r = T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    finally:
        K.cost_volume_supported = sup
    return {n: p.grad.detach().clone() for n, p in r["student"].named_parameters()
            if p.grad is not None}


def main():
    a, b = grads(False), grads(True)
    rows = []
    for n in a:
        d = float((a[n] - b[n]).abs().max()) / (float(b[n].abs().max()) + 1e-30)
        s = abs(float(a[n].double().sum() - b[n].double().sum())) / (float(b[n].double().abs().sum()) + 1e-30)
        rows.append((d, s, n, tuple(a[n].shape)))
    rows.sort(reverse=True)
    for d, s, n, shp in rows[:25]:
        print(f"{d:.2e} (sum {s:.2e}) {n} {shp}")


if __name__ == "__main__":
    main()
