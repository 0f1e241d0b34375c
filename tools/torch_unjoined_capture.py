"""What torch's CUDAGraph.capture_end does on this HIP runtime when a stream forked from the
capture stream still has unjoined work (tools/hip_capture_repro.hip `unjoined`:
hipStreamEndCapture returns hipErrorStreamCaptureUnjoined AND writes a non-null graph
handle).  case `joined` is the control."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libsegv_trace.so"))
assert lib.segv_trace_install() == 0
import torch  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "unjoined"
x = torch.zeros(1024, device="cuda")
side = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
print("case", case, flush=True)
try:
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        x.add_(1)
        side.wait_stream(cap)
        with torch.cuda.stream(side):
            x.mul_(2)
        if case == "joined":
            cap.wait_stream(side)
        if case == "external":  # wait on a stream that is not part of the capture
            idle = torch.cuda.Stream()
            cap.wait_stream(idle)
            cap.wait_stream(side)
            import gc
            gc.collect()
    print("capture_end returned", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replay ok", float(x[0]), flush=True)
except Exception as e:  # noqa: BLE001
    print("raised:", type(e).__name__, str(e)[:300], flush=True)
