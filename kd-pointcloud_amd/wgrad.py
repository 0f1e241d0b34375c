"""Parameter gradients off the backward's critical path.

A layer's backward produces two kinds of output: the gradients of its inputs, which the
next (upstream) backward op waits for, and the gradients of its parameters, which only the
optimizer reads.  The second kind -- the PointConv weight-gradient kernel (pc_bwd_weight,
~1.8 ms of a B=8 training step), the dense layers' split-K weight GEMMs and every bias column
sum -- is issued here on a second HIP stream, forked from the backward's stream at that
point, so it runs beside the rest of the backward instead of in front of it.  Same kernels on
the same inputs: the gradients are bit-identical to issuing them in line.

Ordering (eager and inside a captured HIP graph alike):
  * the side stream waits for the backward's stream before each launch, so it reads finished
    inputs, and the inputs it reads are recorded on it (the caching allocator keeps them
    until it has run);
  * the backward's stream waits for the side stream once, at the end of the backward pass
    (an autograd engine callback), so every `.grad` is complete on that stream when
    backward() returns -- the optimizer step, a gradient pack or a host read that follows
    needs nothing more;
  * code that reads a parameter gradient DURING the backward (a post-accumulate-grad hook,
    e.g. GraphedStep's bucket all-reduces) calls join() first.
`enabled = False` issues everything in line (DDP's reducer reads gradients from its own
hooks during the backward and is not taught to join).
"""
import os

import torch

# KDPC_WGRAD_STREAM=0 issues every parameter gradient in line (A/B runs)
enabled = os.environ.get("KDPC_WGRAD_STREAM", "1") != "0"
_side = {}      # device index -> side stream
_pending = {}   # (main, side) raw stream handles -> (main, side) joins queued in this backward


def side_stream(device):
    s = _side.get(device.index)
    if s is None:
        s = _side[device.index] = torch.cuda.Stream(device=device)
    return s


def run(fn, inputs):
    """fn() launches parameter-gradient kernels reading `inputs` and returns their results;
    run it on the side stream.  Call from inside a torch.autograd.Function.backward."""
    dev = inputs[0].device
    if not enabled or dev.type != "cuda":
        return fn()
    main = torch.cuda.current_stream(dev)
    side = side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:
        if t is not None:
            t.record_stream(side)
    # one join per backward pass: every call queues the (idempotent) callback, the first of
    # them to run at the end of the pass makes `main` wait (a pass that raised and never ran
    # its callbacks leaves nothing stale behind: the next pass queues its own)
    key = (main.cuda_stream, side.cuda_stream)
    _pending[key] = (main, side)
    torch.autograd.Variable._execution_engine.queue_callback(lambda k=key: _join_pending(k))
    return out


def _join_pending(key):
    pair = _pending.pop(key, None)
    if pair is not None:
        pair[0].wait_stream(pair[1])


def join(device=None):
    """The current stream waits for every parameter-gradient kernel issued so far."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    s = _side.get(dev.index)
    if s is not None:
        torch.cuda.current_stream(dev).wait_stream(s)
