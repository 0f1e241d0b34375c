"""Where do the train step's layout copies come from?  One eager FlowTrainStep step under a
TorchDispatchMode that prints every copy of a non-contiguous tensor of >= 256K elements
(aten copy_ / clone / _to_copy / cat inputs) with the project call site.

    python tools/find_copies.py
"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import synthetic  # noqa: E402
from distill import FlowTrainStep, make_optimizer  # noqa: E402
from models_bid_pointconv import PointConvBidirection  # noqa: E402

hits = collections.Counter()


class CopyLog(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = str(func.overloadpacket.__name__)
        if name in ("copy_", "clone", "_to_copy", "contiguous"):
            srcs = [a for a in args if isinstance(a, torch.Tensor)]
            src = srcs[-1] if srcs else None
            if src is not None and src.numel() >= 262144 and not src.is_contiguous():
                st = [f for f in traceback.extract_stack()
                      if "kd-pointcloud_amd" in f.filename and "find_copies" not in f.filename]
                site = " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                                  for f in reversed(st[-3:]))
                hits[(name, tuple(src.shape), tuple(src.stride()), site)] += 1
        return func(*args, **kwargs)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PointConvBidirection().to(dev)
    opt = make_optimizer(model, capturable=True)
    step = FlowTrainStep(model, opt)
    batch = tuple(torch.from_numpy(a).to(dev) for a in synthetic.ft3d_batch(8, 8192, seed=1))
    step(*batch)
    torch.cuda.synchronize()
    with CopyLog():
        step(*batch)
    torch.cuda.synchronize()
    for (name, shape, stride, site), n in sorted(hits.items(), key=lambda kv: -kv[1]):
        print(f"{n:3d} x {name} {shape} stride {stride}\n      {site}")


if __name__ == "__main__":
    main()
