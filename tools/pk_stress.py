"""Packed-f32 stress test (tools/pk_stress.hip): run the packed-vs-scalar
fma chains alone and beside the KD teacher's forward on another stream (the aggressor of the
round-6 race), and count lanes whose packed result differs bit for bit from the scalar one.

  python tools/pk_stress.py [secs=8] [iters=64] [blocks=2048]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
import torch  # noqa: E402

DEV = "cuda"


def main():
    o = dict(a.split("=") for a in sys.argv[1:])
    secs, iters, blocks = float(o.get("secs", 8)), int(o.get("iters", 64)), int(o.get("blocks", 2048))
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "pk_stress.so"))
    lib.pk_stress.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    g = torch.Generator(device="cpu").manual_seed(0)
    n = 4096
    x = (torch.rand(n, generator=g) * 0.5 + 0.1).to(DEV)
    mism = torch.zeros(4, dtype=torch.int64, device=DEV)
    stress = torch.cuda.Stream()

    import synthetic
    from models_bid_pointconv import PointConvBidirection as Teacher
    torch.manual_seed(1)
    teacher = Teacher().to(DEV).eval()
    p1, p2, _ = (torch.from_numpy(a).to(DEV) for a in synthetic.ft3d_batch(4, 8192, seed=31))
    with torch.no_grad():
        plan = teacher.precompute_plan(p1, p2)
        teacher(p1, p2, p1, p2, fps_idx=plan)
    torch.cuda.synchronize()

    def launch(form):
        with torch.cuda.stream(stress):
            rc = lib.pk_stress(form, x.data_ptr(), n, iters, blocks, mism.data_ptr(),
                               stress.cuda_stream)
            assert rc == 0

    lanes = blocks * 256
    for aggressor in (False, True):
        for form in (0, 1):
            mism.zero_()
            torch.cuda.synchronize()
            t0, launches = time.time(), 0
            while time.time() - t0 < secs:
                for _ in range(8):
                    launch(form)
                    launches += 1
                if aggressor:
                    with torch.no_grad():
                        teacher(p1, p2, p1, p2, fps_idx=plan)
                torch.cuda.synchronize()
            bad = int(mism[form])
            ops = launches * lanes * iters * 16 * 4  # packed instructions x 2 lanes each
            print(f"RESULT aggressor={int(aggressor)} form={form} "
                  f"({'op_sel broadcast' if form == 0 else 'no op_sel'}): launches {launches}, "
                  f"lanes {launches * lanes}, packed f32 ops {ops:.3e}, mismatching lanes {bad}",
                  flush=True)


if __name__ == "__main__":
    main()
