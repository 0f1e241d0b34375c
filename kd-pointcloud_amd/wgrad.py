"""Parameter gradients off the backward's critical path.

A layer's backward produces two kinds of output: the gradients of its inputs, which the
next (upstream) backward op waits for, and the gradients of its parameters, which only the
optimizer reads.  The second kind -- the PointConv weight-gradient kernel (pc_bwd_weight,
~1.8 ms of a B=8 training step), the dense layers' split-K weight GEMMs and every bias column
sum -- is issued here on a side HIP stream (_NSTREAMS, round-robin), forked from the backward's
stream at that point, so it runs beside the rest of the backward instead of in front of it.  Same kernels on
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
    e.g. GraphedStep's bucket all-reduces) calls wait_for(params) first: the current stream
    waits for the side-stream event recorded after the launch that produced those
    parameters' gradients (not for everything queued on the side stream so far), or join()
    for all of it;
  * every input of a side-stream launch stays referenced here until that join: autograd's
    InputBuffer adds a second gradient contribution IN PLACE into a gradient tensor it holds
    the only reference to, and AddBackward hands one gradient tensor to both of its inputs, so
    an incoming gradient that run() passed to the side stream could otherwise be modified on
    the backward's stream before the side stream has read it (record_stream only keeps the
    memory from being reused; a held reference keeps the in-place path off);
  * autograd's AccumulateGrad runs on the backward's stream right after the layer's backward
    returns.  With `.grad` None it only takes the new tensor (no kernel reads it), but onto
    an existing `.grad` (accumulation over micro-batches, zero_grad(set_to_none=False)) it
    adds on that stream, reading the side stream's result: run() is told which parameters
    its results are the gradients of, and when any of them already holds a `.grad` the
    backward's stream waits for the side stream at once (the in-line ordering, for that
    layer only).
`enabled = False` issues everything in line; so does any live suspend(owner) (distill.wrap_ddp:
DDP's reducer reads gradients from its own hooks during the backward and is not taught to
join) until its owner is garbage-collected.
"""
import weakref

import torch

# False issues every parameter gradient in line (the tests' bit-identity reference)
enabled = True
# parameter-gradient streams per device, used round-robin by run().  Round 4 measured two
# best (tools/gpu_r4aa.sh: 1 stream 16.07-16.21 ms, 2 streams 15.89-16.04, 3 streams
# 16.01-16.29).  With round 6's kernels one is: train 13.97 -> 13.55 ms, KD 11.13-11.19 ->
# 11.09 (tools/ab_step.py, two runs each, profiles/round06/ab_streams.txt).  The second stream's
# weight kernels competed with the backward for the CUs more than they overlapped each other.
_NSTREAMS = 1
_side = {}      # device index -> the first side stream (the decoder coordinate fork's)
_pool = {}      # device index -> [side streams]
_turn = {}      # device index -> next pool entry
_pending = {}   # (main, side) raw stream handles -> (main, side) joins queued in this backward
_held = {}      # same key -> the side-stream launches' inputs, released at the join
_suspended = weakref.WeakSet()  # objects (DDP wrappers) for whose lifetime run() is in line
# id(leaf parameter) -> (weak reference to it, side-stream event recorded after the launch
# that produced its gradient).  The events stay referenced until overwritten (a HIP event destroyed while a
# graph capture is under way must not be one the capture still tracks).
_ready = {}


def suspend(owner):
    """Issue parameter gradients in line while `owner` is alive."""
    _suspended.add(owner)


def active():
    return enabled and len(_suspended) == 0


def side_stream(device):
    s = _side.get(device.index)
    if s is None:
        s = _side[device.index] = torch.cuda.Stream(device=device)
    return s


def side_streams(device):
    """Every parameter-gradient stream of `device` (the first is side_stream(device))."""
    pool = _pool.get(device.index)
    if pool is None:
        pool = _pool[device.index] = [side_stream(device)] + [
            torch.cuda.Stream(device=device) for _ in range(_NSTREAMS - 1)]
    return pool


def _next_side(device):
    pool = side_streams(device)
    i = _turn.get(device.index, 0)
    _turn[device.index] = (i + 1) % len(pool)
    return pool[i]


def run(fn, inputs, params=()):
    """fn() launches parameter-gradient kernels reading `inputs` and returns their results,
    the gradients of `params`; run it on the side stream.  Call from inside a
    torch.autograd.Function.backward."""
    dev = inputs[0].device
    if not active() or dev.type != "cuda":
        return fn()
    main = torch.cuda.current_stream(dev)
    side = _next_side(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:
        if t is not None:
            t.record_stream(side)
    if params:
        ev = torch.cuda.Event()
        ev.record(side)
        for p in params:
            if p is not None:
                p = _leaf(p)
                _ready[id(p)] = (weakref.ref(p), ev)
    if any(_has_grad(p) for p in params):
        # AccumulateGrad will add onto an existing .grad on `main`: order it after `fn`
        main.wait_stream(side)
        return out
    # one join per backward pass: every call queues the (idempotent) callback, the first of
    # them to run at the end of the pass makes `main` wait (a pass that raised and never ran
    # its callbacks leaves nothing stale behind: the next pass queues its own)
    key = (main.cuda_stream, side.cuda_stream)
    _pending[key] = (main, side)
    _held.setdefault(key, []).append([t for t in inputs if t is not None])
    torch.autograd.Variable._execution_engine.queue_callback(lambda k=key: _join_pending(k))
    return out


def _leaf(p):
    """The parameter behind `p` (the fused layers receive views of their parameters)."""
    while not p.is_leaf and p._base is not None:
        p = p._base
    return p


def _has_grad(p):
    """`p` (a parameter, or a view of one) already holds a .grad."""
    if p is None:
        return False
    p = _leaf(p)
    return p.is_leaf and p.grad is not None


def wait_for(params, stream=None):
    """`stream` (default: the current one) waits for the side-stream launches that produced
    the gradients of `params` -- only those, not the rest of the side stream's queue.
    Parameters whose gradient was produced in line need nothing."""
    seen = set()
    for p in params:
        hit = _ready.get(id(p))
        if hit is None or hit[0]() is not p or id(hit[1]) in seen:
            continue
        seen.add(id(hit[1]))
        (stream or torch.cuda.current_stream(p.device)).wait_event(hit[1])


def _join_pending(key):
    pair = _pending.pop(key, None)
    if pair is not None:
        pair[0].wait_stream(pair[1])
    _held.pop(key, None)


def join(device=None):
    """The current stream waits for every parameter-gradient kernel issued so far."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    for s in _pool.get(dev.index, [s for s in (_side.get(dev.index),) if s is not None]):
        torch.cuda.current_stream(dev).wait_stream(s)
