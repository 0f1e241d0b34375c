"""Model-level gradient error vs float64 (N=2048 trace fixture) under variants of the
cost-volume plumbing (diagnostic): default; batch_prefix replaced by a plain copy (no CSR
derived from the parent index); the unfused wide path.

    python tools/grad_ab2.py
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
    import pointconv_util as P
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    bp, sup = kdpc_native.batch_prefix, kdpc_native.cost_volume_supported
    narrow = lambda din, dout, k: din in (32, 64) and dout in (32, 64) and 1 <= k <= 32  # noqa
    variants = {
        "default": (bp, sup),
        "prefix-copy": (lambda idx, b: idx[:b].clone(), sup),
        "unfused-wide": (bp, narrow),
        "unfused-wide+prefix-copy": (lambda idx, b: idx[:b].clone(), narrow),
    }
    for tag, (bpf, supf) in variants.items():
        kdpc_native.batch_prefix, kdpc_native.cost_volume_supported = bpf, supf
        P._nat.batch_prefix = bpf
        try:
            routing = T._AmaxReplay(g64)
            r = T._run_models(g, T._KnnReplay(g), routing)
            rel, pre = T._grad_errors(r["student"], g, g64)
        finally:
            kdpc_native.batch_prefix, kdpc_native.cost_volume_supported = bp, sup
            P._nat.batch_prefix = bp
        worst = sorted(((e, n) for n, e in rel.items()), reverse=True)[:4]
        print(f"{tag:26s}", "  ".join(f"{e:.2e} {n}" for e, n in worst), flush=True)


if __name__ == "__main__":
    main()
