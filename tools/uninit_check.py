"""Uninitialised-read detector (diagnostic): fill the caching allocator's free memory with
NaN, run the model's forward + KD backward on the N=2048 trace fixture, and report the first
kdpc_native op whose outputs hold NaN while its tensor inputs do not.

    python tools/uninit_check.py
"""
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _tensors(x):
    if torch.is_tensor(x):
        yield x
    elif isinstance(x, (list, tuple)):
        for y in x:
            yield from _tensors(y)
    elif hasattr(x, "offsets"):  # Csr
        yield x.offsets
        yield x.perm


def _has_nan(ts):
    return any(t.is_floating_point() and bool(torch.isnan(t).any()) for t in ts)


def main():
    import kdpc_native as K
    import test_gpu_model as T
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    g64 = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048_f64.npz"))
    hits = []
    skip = {"load_library", "set_launch_timer", "LaunchTimer", "Csr", "attach_csr"}
    for name in dir(K):
        fn = getattr(K, name)
        if name.startswith("_") or name in skip or not callable(fn) or isinstance(fn, type):
            continue
        if getattr(fn, "__module__", None) != K.__name__:
            continue

        def wrap(f, nm):
            @functools.wraps(f)
            def w(*a, **k):
                out = f(*a, **k)
                ins = list(_tensors(list(a) + list(k.values())))
                outs = list(_tensors(out))
                if outs and not _has_nan(ins) and _has_nan(outs):
                    hits.append((nm, [tuple(t.shape) for t in outs if t.is_floating_point()
                                      and bool(torch.isnan(t).any())]))
                return out
            return w
        setattr(K, name, wrap(fn, name))
    junk = torch.full((6 << 30,), float("nan"), device="cuda")  # 24 GB of NaN, then cached
    del junk
    r = T._run_models(g, T._KnnReplay(g), T._AmaxReplay(g64))
    torch.cuda.synchronize()
    nan_params = [n for n, p in r["student"].named_parameters()
                  if p.grad is not None and bool(torch.isnan(p.grad).any())]
    print("first NaN-producing ops:", hits[:10])
    print("params with NaN grads:", len(nan_params), nan_params[:10])
    rel, pre = T._grad_errors(r["student"], g, g64)
    worst = sorted(((e, n) for n, e in rel.items()), reverse=True)[:4]
    print("worst grad errors:", worst)


if __name__ == "__main__":
    main()
