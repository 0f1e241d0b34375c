"""A/B of the model-level gradient errors vs the float64 reference (N=2048 trace fixture)
with the fused wide cost volume (D = 128/256 through kdpc_cost_volume_*) and with the
unfused wide path forced (diagnostic).

    python tools/grad_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    import kdpc_native
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    new = kdpc_native.cost_volume_supported
    old = lambda din, dout, k: din in (32, 64) and dout in (32, 64) and 1 <= k <= 32  # noqa: E731
    for tag, fn in (("fused", new), ("unfused-wide", old)):
        kdpc_native.cost_volume_supported = fn
        routing = T._AmaxReplay(g64)
        r = T._run_models(g, T._KnnReplay(g), routing)
        rel, pre = T._grad_errors(r["student"], g, g64)
        worst = sorted(((e, n) for n, e in rel.items()), reverse=True)[:8]
        print(tag, "changed routing", routing.changed, routing.per_call)
        for e, n in worst:
            print(f"   {e:.3e} {n}")
    kdpc_native.cost_volume_supported = new


if __name__ == "__main__":
    main()
