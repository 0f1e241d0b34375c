"""Cost-volume forward (D <= 64) at the model's narrow calls (B=16 pair batch): HIP events,
kernel only; output checksums printed so a restructured kernel can be checked bit for bit.

    python tools/bench_cv_fwd.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402

DEV = "cuda"
SHAPES = {"cross0 (B16 N8192 K32 D32)": (16, 8192, 32, 32, 32),
          "cross1 (B16 N2048 K32 D64)": (16, 2048, 32, 64, 64)}


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (B, N, Kn, di, do) in SHAPES.items():
        x1 = torch.rand(B, N, 3, generator=g).to(DEV)
        x2 = torch.rand(B, N, 3, generator=g).to(DEV)
        idx = K.knn_point(Kn, x2, x1)
        p1 = torch.randn(B, N, di, generator=g).to(DEV)
        p2 = torch.randn(B, N, di, generator=g).to(DEV)
        wpos = torch.randn(di, 3, generator=g).to(DEV)
        bpos = torch.randn(di, generator=g).to(DEV)
        w1 = (torch.randn(do, di, generator=g) / di ** 0.5).to(DEV)
        b1 = torch.randn(do, generator=g).to(DEV)
        f = lambda: K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)  # noqa: E731
        out0 = f()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            f()
        e.record()
        torch.cuda.synchronize()
        print(name, "us",
              round(s.elapsed_time(e) / 20 * 1e3, 1),
              "checksum", float(out0[0].double().sum()), int(out0[1].long().sum()), flush=True)


if __name__ == "__main__":
    main()
