"""Fused vs unfused wide cost volume: the gradient arriving at every dense (Linear / 1x1) layer
output and every cost-volume output in two full model runs (N=2048 trace fixture, float64
routing replayed), listed in backward order (diagnostic).

    python tools/lin_gout_ab.py
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
    import dense
    import kdpc_native as K
    import pointconv_util as P
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    sup = K.cost_volume_supported
    if narrow_only:
        K.cost_volume_supported = lambda din, dout, k: din in (32, 64) and dout in (32, 64)
    fwd, order = [], []
    targets = [(dense._Linear, "lin"), (P._CostVolume, "cv"), (P._CostVolumeWide, "cv")]
    origs = [t.apply for t, _ in targets]

    def wrap(orig, tag):
        def f(*a):
            out = orig(*a)
            i = len(fwd)
            fwd.append((tag, tuple(out.shape), out.detach().clone()))
            if out.requires_grad:
                def hook(gr, i=i):
                    order.append((i, gr.detach().clone()))
                out.register_hook(hook)
            return out
        return f
    for (t, tag), o in zip(targets, origs):
        t.apply = wrap(o, tag)
    try:
        T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    finally:
        for (t, _), o in zip(targets, origs):
            t.apply = o
        K.cost_volume_supported = sup
    torch.cuda.synchronize()
    return fwd, order


def main():
    fa, oa = run(False)
    fb, ob = run(True)
    print("forward calls", len(fa), len(fb), "hooked grads", len(oa), len(ob))
    gb = dict(ob)
    for i, ga in oa:
        tag, shp, _ = fa[i]
        if i not in gb:
            continue
        b = gb[i]
        d = float((ga - b).abs().max()) / (float(b.abs().max()) + 1e-30)
        fo = float((fa[i][2] - fb[i][2]).abs().max()) / (float(fb[i][2].abs().max()) + 1e-30)
        flag = " <==" if d > 1e-5 else ""
        print(f"fwd#{i:3d} {tag:3s} {shp}: out rel {fo:.1e}  grad rel {d:.2e}{flag}", flush=True)


if __name__ == "__main__":
    main()
