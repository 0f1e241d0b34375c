"""Fused vs unfused wide cost volume inside the model run (N=2048 trace fixture, float64 max
routing replayed): the forward output and the incoming gradient of every cost-volume call,
run against run (diagnostic).

    python tools/cv_gout_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(narrow_only):
    import kdpc_native as K
    import pointconv_util as P
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    sup = K.cost_volume_supported
    if narrow_only:
        K.cost_volume_supported = lambda din, dout, k: din in (32, 64) and dout in (32, 64)
    outs, gouts = [], []
    fns = (P._CostVolume, P._CostVolumeWide)
    origs = [f.apply for f in fns]

    def wrap(orig):
        def f(*a):
            out = orig(*a)
            i = len(outs)
            outs.append(out.detach().clone())
            gouts.append(None)
            if out.requires_grad:
                def hook(gr, i=i):
                    gouts[i] = gr.detach().clone()
                out.register_hook(hook)
            return out
        return f
    for fn, o in zip(fns, origs):
        fn.apply = wrap(o)
    try:
        r = T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    finally:
        for fn, o in zip(fns, origs):
            fn.apply = o
        K.cost_volume_supported = sup
    torch.cuda.synchronize()
    return outs, gouts


def main():
    a_out, a_g = run(False)
    b_out, b_g = run(True)
    for i, (ao, bo, ag, bg) in enumerate(zip(a_out, b_out, a_g, b_g)):
        s = f"call {i:2d} {tuple(ao.shape)}: out rel {float((ao - bo).abs().max()) / float(bo.abs().max()):.2e}"
        if ag is not None and bg is not None:
            s += f"  gout rel {float((ag - bg).abs().max()) / (float(bg.abs().max()) + 1e-30):.2e}"
        print(s, flush=True)


if __name__ == "__main__":
    main()
