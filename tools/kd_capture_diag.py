"""Diagnose the HIP-graph capture of the KD step with the student's decoder coordinate fork
(round-3 segfault in capture_end).  One capture per process:

    KDPC_KD_COORD_FORK=1 python tools/kd_capture_diag.py [--keep-events] [--n 2048]

--keep-events keeps every torch.cuda.Event created during the capture alive until after
capture_end (tests whether an event destroyed mid-capture is what the runtime trips over).
A native backtrace handler (tools/libsegv_trace.so) prints the C frames of a crash."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--keep-events", action="store_true")
ap.add_argument("--n", type=int, default=2048)
ap.add_argument("--b", type=int, default=2)
ap.add_argument("--replays", type=int, default=3)
ap.add_argument("--seq", action="store_true",
                help="run tests/test_gpu_graph.py::test_graphed_step_equals_eager[train] then "
                     "[kd] in this process (the round-3 crash sequence)")
args = ap.parse_args()

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libsegv_trace.so"))
assert lib.segv_trace_install() == 0

import torch  # noqa: E402

if args.keep_events:
    _kept = []
    _orig_record = torch.cuda.Stream.record_event

    def record_event(self, event=None):
        ev = _orig_record(self, event)
        _kept.append(ev)
        return ev
    torch.cuda.Stream.record_event = record_event

import distill  # noqa: E402
import synthetic  # noqa: E402
from models_bid_pointconv import PointConvBidirection  # noqa: E402

print(f"KD_COORD_FORK={distill.KD_COORD_FORK} TEACHER_STREAM={distill.TEACHER_STREAM} "
      f"keep_events={args.keep_events}", flush=True)
if args.seq:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_gpu_graph as T
    for mode in ("train", "kd"):
        T.test_graphed_step_equals_eager(mode)
        print(f"SEQ {mode} OK", flush=True)
    sys.exit(0)
dev = "cuda"
torch.manual_seed(0)
student = PointConvBidirection().to(dev)
teacher = PointConvBidirection().to(dev)
opt = distill.make_optimizer(student, capturable=True)
b = tuple(torch.from_numpy(a).to(dev) for a in synthetic.ft3d_batch(args.b, args.n, seed=1))
step = distill.graphed_kd_step(teacher, student, opt, b, warmup=1)
print("CAPTURE OK", flush=True)
for _ in range(args.replays):
    loss = step(*b, next_batch=b)
torch.cuda.synchronize()
print(f"REPLAY OK loss={float(loss):.6f}", flush=True)
