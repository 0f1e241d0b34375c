"""Training and knowledge-distillation steps, single GPU or DDP over RCCL.

Restates the per-step body of distilTrain.py:156-185 (and the flow-network step of
train_bid_pointconv.py) MI355X-first:
  * one process per GPU, torch DDP (backend "nccl" = RCCL over xGMI) instead of the
    reference's single-process nn.DataParallel (distilTrain.py:108-117).  DDP's bucketed
    gradient all-reduce runs on RCCL's own stream, overlapped with the backward;
  * the frozen teacher is replicated per rank outside DDP (no communication);
  * BatchNorm statistics stay per replica (the DataParallel semantics, no SyncBN);
    broadcast_buffers keeps rank 0's running stats authoritative, as DataParallel's
    device-0 module was;
  * the 80 parameters that never receive a gradient (the cost volumes' unused
    bias1/bias2, WeightNet's unused BN modules) are handled by static_graph;
  * no per-step host sync: the loss stays on the device (the reference called
    loss.cpu() twice per step, distilTrain.py:179,184).
The step is model-agnostic (any module returning the reference's 8-tuple), which lets the
multi-process path be tested on CPU with gloo.
"""

import os

import torch
import torch.distributed as dist

import kdpc_native as _nat
import loss_functions
import wgrad


def is_dist():
    return dist.is_available() and dist.is_initialized()


def wrap_ddp(model, device=None):
    """Wrap the trained model for DDP when a process group is up (no-op otherwise).

    DDP's reducer reads each gradient from its own hook during the backward, so while a DDP
    wrapper made here is alive the parameter gradients are issued in line (wgrad.py:
    wgrad.suspend(), released when the wrapper is garbage-collected)."""
    if not is_dist() or dist.get_world_size() == 1:
        return model
    kw = dict(broadcast_buffers=True, static_graph=True, gradient_as_bucket_view=True)
    if device is not None and device.type == "cuda":
        kw["device_ids"] = [device.index]
    ddp = torch.nn.parallel.DistributedDataParallel(model, **kw)
    wgrad.suspend(ddp)
    return ddp


def make_optimizer(model, lr=1e-3, weight_decay=1e-4, capturable=False):
    """Adam as configured by config_train_kd_pointconv.yaml:15-24 / distilTrain.py:134-135.
    capturable=True keeps the step counters on the device (required by GraphedStep).  On
    the GPU the fused (single multi-tensor kernel) implementation is used: the same Adam
    update (L2 weight decay, not AdamW) in one launch instead of ~10 foreach passes."""
    params = list(model.parameters())
    fused = len(params) > 0 and all(p.is_cuda for p in params)
    if capturable and fused:
        # a device tensor: a graph replay reads it, so LR changes reach the captured update
        lr = torch.tensor(float(lr), device=params[0].device)
    return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-08,
                            weight_decay=weight_decay, capturable=capturable,
                            fused=True if fused else None)


# the graphed step's flat Adam on csrc/adam.hip (one launch) rather than torch's fused Adam
# (multi-tensor, 7 launches); both give the same bits (tests/test_gpu_adam.py)
HIP_ADAM = True


def _core(model):
    return model.module if isinstance(model, torch.nn.parallel.DistributedDataParallel) else model


# True runs the frozen teacher's forward on a stream of its own, beside the student's forward
# (round 3: 15.6 -> 13.8 ms per KD step), eagerly through _TeacherFork and in the graphed step.
# Round 5 switched it off because graphed KD steps disagreed now and then; round 6 found why
# (DESIGN §5): packed f32 instructions (v_pk_fma_f32 ...) gave wrong results now and then
# while the other stream's kernels ran beside them.  The library holds none since, and the
# two-stream step is bit-reproducible.  The teacher and the student share the coordinate
# plan (no private copy: nothing of it is written by either).
TEACHER_STREAM = True
# the graphed KD step: the teacher's forward as a graph of its own on the teacher stream,
# beside the student's forward graph (True), or as a concurrent branch of the one step graph
# (False).  KDPC_TEACHER_GRAPH=0/1 overrides (A/B runs).
TEACHER_GRAPH = os.environ.get("KDPC_TEACHER_GRAPH", "0") == "1"
_teacher_streams = {}


def _teacher_stream(dev):
    s = _teacher_streams.get(dev.index)
    if s is None:
        s = _teacher_streams[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _detached(x):
    if isinstance(x, torch.Tensor):
        return x.detach()
    if isinstance(x, (list, tuple)):
        return type(x)(_detached(t) for t in x)
    return x


class _TeacherFork:
    """The frozen teacher's forward (no_grad) on its own stream, beside the student's forward:
    the two share only their inputs, and at B=4 per GPU neither fills the chip.  join()
    makes the current stream wait before the teacher's outputs are read (the KD loss).  Same
    kernels on the same inputs: bit-identical to running the teacher in line.  Inside a graph
    capture the fork becomes a concurrent branch of the captured graph."""

    def __init__(self, teacher, args, kw):
        dev = args[0].device
        self.cur = self.side = None
        if TEACHER_STREAM and dev.type == "cuda":
            self.cur = torch.cuda.current_stream(dev)
            self.side = _teacher_stream(dev)
            self.side.wait_stream(self.cur)
            with torch.cuda.stream(self.side), torch.no_grad():
                self.out = teacher(*args, **kw)
        else:
            with torch.no_grad():
                self.out = teacher(*args, **kw)

    def join(self):
        if self.side is not None:
            self.cur.wait_stream(self.side)
        return self.out


# True: the KD student forks its decoder searches too (measured slower; tests)
KD_COORD_FORK = False


class _kd_student_streams:
    """Context for the KD student's forward.  The KD step already runs the teacher's forward
    on a stream of its own, beside the student's; there the student's decoder coordinate fork
    (models_bid_pointconv._CoordFork) measured slower, with its own stream (13.17-13.66 vs
    14.27-14.30 ms/step at configs[3]'s slice, profiles/round03/ab/bab_fkkd_*) and on the
    parameter-gradient stream alike (13.56-13.66 vs 14.30-14.32, bab_fskd_*), so the student
    searches in line inside the KD step (KD_COORD_FORK = True keeps the fork).  Scoped to
    the step's own forward: the same module trained by a FlowTrainStep keeps its fork."""

    def __init__(self, student):
        core = _core(student)
        self.core = core if (hasattr(core, "coord_fork") and not KD_COORD_FORK) else None

    def __enter__(self):
        if self.core is not None:
            self.prev = self.core.__dict__.get("coord_fork")
            self.core.coord_fork = False
        return self

    def __exit__(self, *exc):
        if self.core is not None:
            if self.prev is None:
                del self.core.coord_fork  # back to the class default
            else:
                self.core.coord_fork = self.prev
        return False


def _plan_fn(model):
    """The model's coordinate-only precompute: the FPS chain plus the coordinate-only kNN
    searches and their CSRs (PointConvBidirection.precompute_plan) where the model has it,
    else the FPS chain alone."""
    return getattr(model, "precompute_plan", None) or model.precompute_fps


class FpsPrefetch:
    """Runs the encoder's FPS chain, the coordinate-only kNN searches and their CSRs
    (PointConvBidirection.precompute_plan) for an upcoming batch on a side HIP stream.  FPS
    is one workgroup per cloud for ~2900 dependent steps (2.5 ms per B=8 step,
    latency-bound on 16 CUs); issued one step ahead it runs beside the current step's
    kernels instead of in front of them, and the 13 searches that depend on coordinates only
    run after it on the same stream.  Results are identical to computing them inside the
    forward (same kernels, same inputs)."""

    def __init__(self):
        self.stream = None
        self.inputs = None  # strong references: identity, not a reusable address, is the key
        self.fps = None
        self.event = None

    @staticmethod
    def _versions(pos1, pos2):
        return (pos1._version, pos2._version)

    def launch(self, model, pos1, pos2):
        if not pos1.is_cuda:
            return
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=pos1.device)
        self.stream.wait_stream(torch.cuda.current_stream(pos1.device))
        with torch.cuda.stream(self.stream):
            self.fps = _plan_fn(_core(model))(pos1, pos2)
            self.event = torch.cuda.Event()
            self.event.record(self.stream)
        # the side stream reads pos1/pos2: keep the caching allocator from handing their
        # blocks to the main stream before the FPS chain has finished with them
        pos1.record_stream(self.stream)
        pos2.record_stream(self.stream)
        self.inputs = (pos1, pos2, self._versions(pos1, pos2))

    def take(self, pos1, pos2):
        """The prefetched indices if they were computed for exactly these (unmodified)
        tensor objects."""
        if self.fps is None or self.inputs is None:
            return None
        p1, p2, ver = self.inputs
        if p1 is not pos1 or p2 is not pos2 or ver != self._versions(pos1, pos2):
            return None
        cur = torch.cuda.current_stream(pos1.device)
        cur.wait_event(self.event)
        for t in self.fps:
            t.record_stream(cur)
        fps, self.fps, self.inputs = self.fps, None, None
        return fps


class FlowTrainStep:
    """fwd -> multiScaleLoss -> bwd -> optimizer step (one scene-flow training iteration)."""

    def __init__(self, model, optimizer, loss_fn=None):
        self.model = model
        self.opt = optimizer
        self.loss_fn = loss_fn or loss_functions.multiScaleLoss
        self.prefetch = FpsPrefetch()

    def __call__(self, pos1, pos2, flow, color1=None, color2=None, next_batch=None):
        """next_batch: optional (pos1, pos2, ...) of the following step; its FPS is issued
        on a side stream now (FpsPrefetch)."""
        color1 = pos1 if color1 is None else color1
        color2 = pos2 if color2 is None else color2
        fps = self.prefetch.take(pos1, pos2)
        if next_batch is not None:
            self.prefetch.launch(self.model, next_batch[0], next_batch[1])
        self.model.train()
        kw = {} if fps is None else {"fps_idx": fps}
        flows, fps1, _, _, _, _, _, _ = self.model(pos1, pos2, color1, color2, **kw)
        loss = self.loss_fn(flows, flow, fps1)
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        return loss.detach()


class KDTrainStep:
    """distilTrain.py:164-182: teacher fwd (eval, no_grad) + student fwd (train) + KD loss +
    bwd + step.  The loss is biDirection_loss_ht(gamma=0.3, beta=0.8, layer=3): the shipped
    cross_biDirection_loss_ht cannot run on this teacher/student pair."""

    def __init__(self, teacher, student, optimizer, gamma=0.3, beta=0.8, layer=3, loss_fn=None):
        self.loss_fn = loss_fn or loss_functions.biDirection_loss_ht
        self.teacher = teacher
        self.student = student
        self.opt = optimizer
        self.gamma, self.beta, self.layer = gamma, beta, layer
        self.prefetch = FpsPrefetch()
        for p in self.teacher.parameters():
            p.requires_grad_(False)

    def __call__(self, pos1, pos2, flow, color1=None, color2=None, next_batch=None):
        color1 = pos1 if color1 is None else color1
        color2 = pos2 if color2 is None else color2
        fps = self.prefetch.take(pos1, pos2)
        if fps is None and pos1.is_cuda:  # teacher and student share one FPS chain
            fps = _plan_fn(_core(self.student))(pos1, pos2)
        if next_batch is not None:
            self.prefetch.launch(self.student, next_batch[0], next_batch[1])
        kw = {} if fps is None else {"fps_idx": fps}
        self.teacher.eval()
        t_fork = _TeacherFork(self.teacher, (pos1, pos2, color1, color2), kw)
        self.student.train()
        with _kd_student_streams(self.student):
            flows, fps1, fps2, _, _, feat1s, feat2s, _ = self.student(pos1, pos2, color1,
                                                                      color2, **kw)
        t_flows, t_fps1, t_fps2, _, _, t_feat1s, t_feat2s, _ = t_fork.join()
        loss = self.loss_fn(
            flows, feat1s, feat2s, fps1, fps2, flow, t_flows, t_feat1s, t_feat2s, t_fps1, t_fps2,
            self.gamma, self.beta, layer=self.layer)
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        return loss.detach()


@torch.no_grad()
def epe3d(model, pos1, pos2, flow):
    """EPE3D as distilTrain.py:229 / evaluation_utils.py:23-24: mean ||flow0^T - gt||."""
    model.eval()
    flows = model(pos1, pos2, pos1, pos2)[0]
    return torch.norm(flows[0].permute(0, 2, 1) - flow, dim=2).mean()


def _capturing(stream):
    with torch.cuda.stream(stream):
        return torch.cuda.is_current_stream_capturing()


def _join_capture_streams(cap, extra=()):
    """Make the capture stream wait for every side stream this process forks from a capture
    (the plan fork, the all-reduce stream, the parameter-gradient stream, the teacher's
    stream, the decoder coordinate forks) that is still part of the capture.  Every code path
    joins its streams already; this is the guarantee: on this HIP runtime a capture that ends
    with unjoined work on a forked stream does not fail cleanly -- hipStreamEndCapture
    returns hipErrorStreamCaptureUnjoined but still writes a graph handle, and torch's
    capture_end then crashed in the round-3 KD capture (DESIGN §5,
    tools/hip_capture_repro.hip `unjoined`, tools/torch_unjoined_capture.py).  Waiting on a
    stream whose work is already joined adds no work."""
    import models_bid_pointconv
    dev = cap.device
    streams = [s for s in extra if s is not None]
    streams += list(wgrad._pool.get(dev.index, [wgrad._side.get(dev.index)]))
    streams += [_teacher_streams.get(dev.index)]
    streams += [s for (d, _), s in models_bid_pointconv._coord_streams.items() if d == dev.index]
    seen = set()
    for s in streams:
        if s is None or s.cuda_stream in seen or s.cuda_stream == cap.cuda_stream:
            continue
        seen.add(s.cuda_stream)
        if _capturing(s):
            cap.wait_stream(s)


class GraphedStep:
    """One training step replayed from HIP graphs (MI355X: the eager step issues ~2000
    launches per iteration from Python, as much host time as the GPU needs).

    world 1:  ONE graph = [FPS of the NEXT batch on a forked stream] + forward + loss +
              backward + gradient pack + flat Adam step.
    world > 1, RCCL (`nccl` backend; one process per GPU over xGMI) -- "overlap" schedule:
              still ONE graph.  The gradients are packed, in the order the backward
              finalises them, into buckets of about `bucket_bytes`; as soon as the backward
              has produced a bucket it is all-reduced on a side stream forked from the
              capture (RCCL kernels captured into the graph), beside the rest of the
              backward; the main stream joins the side stream before the mean + flat Adam.
              DDP's overlap, without DDP's per-step host work.
    world > 1, other backends (gloo cannot be captured) -- "serial" schedule: graph A (fwd +
              bwd + pack), one eager all-reduce of the flat gradient, graph B (mean + Adam).
    The averaged-gradient semantics are DDP's (and the reference DataParallel's): every
    replica applies the same Adam update to the mean gradient.

    Optimizer: the trained parameters (and Adam's moments) become views of flat buffers laid
    out in gradient-ready order, updated by ONE fused Adam over all 8 M values.  The caller's
    optimizer keeps working on the same storage: its per-parameter `step` counters are
    copied from the flat counter inside the graph (and the flat counter from them before
    each update, so eager steps in between are honoured), and the learning rate is one
    device tensor shared by both optimizers -- an LR scheduler (or a plain
    `param_groups[0]['lr'] = x`, re-read before every replay) reaches the graph.  After the
    capture the parameters' `.grad` are None again (the graph keeps its own buffers), so an
    eager step in between starts from empty gradients as it would without the graph.

    `loss_fn(*inputs)` must run the whole forward (model call(s) and loss) and return the
    loss; the inputs are copied into static buffers before each replay.  Warm-up iterations
    run eagerly on a side stream (they allocate lazily-initialised state: optimizer moments,
    cached attributes, the communicator).

    prefetch_fn (optional, e.g. PointConvBidirection.precompute_plan): a function of the first
    `n_prefetch` inputs whose result loss_fn takes as `fps=`.  The graph then runs it for the
    next batch on a forked stream, beside this batch's forward/backward, into buffers the next
    replay reads.  A call whose batch is not the previous call's `next_batch` recomputes it
    eagerly first, so results never depend on what was prefetched.

    overlap: None = "overlap" schedule when world > 1 and the backend is nccl (RCCL);
    True forces it (also at world 1, where the all-reduces are one-rank collectives: the
    capture mechanics test); False forces "serial"."""

    drop_warmup_graph = True  # diagnostics seam (tools/graph_diag.py)
    capture_on_side_stream = False
    bucket_bytes = 8 << 20  # all-reduce bucket size (world > 1)

    def __init__(self, loss_fn, params, optimizer, example_inputs, warmup=3, prefetch_fn=None,
                 n_prefetch=2, overlap=None, stages=None):
        if warmup < 1:
            raise ValueError("GraphedStep needs warmup >= 1: the last warm-up backward records "
                             "the gradient order the flat buffers are laid out in")
        self.loss_fn = loss_fn
        # stages = (side_fn, forward_fn, loss_from): the step as three captured graphs (see
        # _capture_stages); loss_fn stays the eager form, used by the warm-up iterations
        self.stages = stages
        self.opt = optimizer
        self.params = [p for p in params if p.requires_grad]
        self.static = [t.detach().clone() for t in example_inputs]
        self.world = dist.get_world_size() if is_dist() else 1
        if overlap is None:
            overlap = self.world > 1 and dist.get_backend() == "nccl"
        if overlap and not is_dist():
            raise ValueError("GraphedStep(overlap=True) needs an initialised process group")
        self.schedule = "overlap" if overlap else ("serial" if self.world > 1 else "single")
        self.prefetch_fn = prefetch_fn
        self.n_prefetch = n_prefetch
        self.static_next = [t.detach().clone() for t in example_inputs[:n_prefetch]]
        self._pending = None  # (tensors, versions) the buffered prefetch was computed for
        self._check_optimizer()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        order = []
        with torch.cuda.stream(side):
            loss = None
            for i in range(warmup):
                self.opt.zero_grad(set_to_none=True)
                loss = self.loss_fn(*self.static, **self._fps_kw(self._eager_prefetch()))
                hooks = ([p.register_post_accumulate_grad_hook(order.append)
                          for p in self.params] if i == warmup - 1 else [])
                loss.backward()
                for h in hooks:
                    h.remove()
                self._allreduce_eager()
                self.opt.step()
            # drop the last warm-up graph: while it lives, the parameters' AccumulateGrad
            # nodes (created on this side stream) would be reused by the captured backward
            if self.drop_warmup_graph:
                del loss
            self.fps_cur = self._eager_prefetch()
            if self.fps_cur is not None:
                self.fps_cur = [t.clone() for t in self.fps_cur]
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._flat_adam(order)
        self.opt.zero_grad(set_to_none=True)
        self.graph_a = torch.cuda.CUDAGraph()
        kw = {"stream": side} if self.capture_on_side_stream else {}
        if self.world > 1 or self.schedule == "overlap":
            # a process group's background threads (RCCL watchdog: event queries) may touch the
            # runtime while this thread captures; "global" mode would fail those calls
            kw["capture_error_mode"] = "thread_local"
        fork = torch.cuda.Stream() if prefetch_fn is not None else None
        self.comm = torch.cuda.Stream() if self.schedule == "overlap" else None
        self.graph_t = self.graph_f = None
        if self.stages is not None:
            self._capture_stages(kw, fork)
        hooks = self._bucket_hooks() if self.schedule == "overlap" else []
        kw_a = dict(kw, pool=self.graph_f.pool()) if self.stages is not None else kw
        with torch.cuda.graph(self.graph_a, **kw_a):
            cap = torch.cuda.current_stream()
            self._cap = cap
            if fork is not None and self.stages is None:
                # the previous replay's tail copied its fps_next into fps_cur
                fork.wait_stream(cap)
                with torch.cuda.stream(fork):
                    self.fps_next = list(prefetch_fn(*self.static_next))
            if self.stages is None:
                self.loss = self.loss_fn(*self.static, **self._fps_kw(self.fps_cur))
            else:  # the loss of the captured forward stage and the teacher graph's outputs
                self.loss = self.stages[2](self.s_out, self.t_out, *self.static)
            self.loss.backward()
            if fork is not None and self.stages is None:
                cap.wait_stream(fork)
            if self.schedule == "overlap":
                cap.wait_stream(self.comm)  # every bucket's all-reduce
                if self.world > 1:
                    self.G.div_(float(self.world))
                self._tail(fork, pack=False)
            elif self.schedule == "single":
                self._tail(fork)
            else:  # serial: pack only; the all-reduce runs between graph A and graph B
                self._pack()
            _join_capture_streams(cap, (fork, self.comm))
        for h in hooks:
            h.remove()
        if self.schedule == "overlap" and any(not b["done"] for b in self.buckets):
            raise RuntimeError("GraphedStep: a gradient bucket was never completed in capture")
        self.graph_b = None
        if self.schedule == "serial":
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b, pool=self.graph_a.pool(), **kw):
                self.G.div_(float(self.world))
                self._tail(fork, pack=False)
        torch.cuda.synchronize()
        # the graph owns its gradient buffers; the parameters' .grad go back to None so an
        # eager step in between does not accumulate onto the last replay's gradients
        self._grad_refs = [p.grad for p in self.params]
        for p in self.params:
            p.grad = None
        # keep the static loss buffer, not the captured autograd graph: while that graph
        # lives, an eager step on the same parameters reuses its AccumulateGrad nodes (bound
        # to the capture stream) and torch warns of a stream mismatch (bench's eager
        # measurement steps after the timed region)
        self.loss = self.loss.detach()
        if self.stages is not None:  # the forward stage's outputs, without its autograd graph
            self.s_out = _detached(self.s_out)
        self._pending = None

    def _capture_stages(self, kw, fork):
        """stages = (side_fn, forward_fn, loss_from): side_fn (the KD step's frozen teacher
        forward, no_grad) is captured as a graph of its own on the teacher stream, forward_fn
        (the student forward, with the next batch's coordinate plan on the forked stream) as a
        second graph on the capture stream; the caller then captures loss_from(forward out,
        side out, *inputs) + backward + optimizer as graph_a in the forward graph's pool (it
        reads the forward's saved tensors).  A replay runs the first two side by side on two
        streams and joins them before graph_a.  (Round 6 added this form while chasing the
        multi-stream race, whose cause was packed f32 instructions; it is
        bit-identical to the one-graph form and 0.3 ms slower, so it is the option
        TEACHER_GRAPH, not the default.)"""
        side_fn, fwd_fn, _ = self.stages
        cur = torch.cuda.current_stream()
        ts = _teacher_stream(self.static[0].device)
        self.graph_t = torch.cuda.CUDAGraph()
        ts.wait_stream(cur)
        kwt = {k: v for k, v in kw.items() if k != "stream"}
        with torch.cuda.graph(self.graph_t, stream=ts, **kwt):
            with torch.no_grad():
                self.t_out = side_fn(*self.static, **self._fps_kw(self.fps_cur))
        cur.wait_stream(ts)
        self.graph_f = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_f, **kw):
            cap = torch.cuda.current_stream()
            if fork is not None:
                fork.wait_stream(cap)  # the previous replay's tail wrote fps_cur
                with torch.cuda.stream(fork):
                    self.fps_next = list(self.prefetch_fn(*self.static_next))
            self.s_out = fwd_fn(*self.static, **self._fps_kw(self.fps_cur))
            if fork is not None:
                cap.wait_stream(fork)
            _join_capture_streams(cap, (fork,))

    def _replay(self):
        if self.graph_t is not None:
            cur = torch.cuda.current_stream()
            ts = _teacher_stream(self.static[0].device)
            ts.wait_stream(cur)  # the static inputs and the plan are written on `cur`
            with torch.cuda.stream(ts):
                self.graph_t.replay()
            self.graph_f.replay()
            cur.wait_stream(ts)
        self.graph_a.replay()

    def schedule_name(self):
        if self.graph_t is not None:
            return (" (3 graphs: teacher fwd on its own stream beside the student fwd, then "
                    "loss+bwd+flat Adam" + (", bucketed all-reduces" if self.schedule == "overlap"
                                            else "") + ")")
        if self.schedule == "single":
            return " (1 graph: fwd+bwd+flat Adam)"
        if self.schedule == "overlap":
            return (f" (1 graph: fwd+bwd with {len(self.buckets)} gradient buckets all-reduced "
                    "on a captured side stream as the backward completes them, then flat Adam)")
        return " (graph A fwd+bwd -> eager flat all-reduce -> graph B flat Adam)"

    def _check_optimizer(self):
        opt = self.opt
        ok = type(opt) is torch.optim.Adam and len(opt.param_groups) == 1
        grp = opt.param_groups[0] if ok else {}
        if not (ok and grp.get("fused") and grp.get("capturable") and not grp.get("amsgrad")):
            raise ValueError("GraphedStep needs a single-group torch.optim.Adam with fused=True, "
                             "capturable=True (distill.make_optimizer(..., capturable=True))")
        ids = {id(p) for p in self.params}
        if {id(p) for p in grp["params"] if p.requires_grad} != ids:
            raise ValueError("GraphedStep: the optimizer must hold exactly the trained parameters")

    def _flat_adam(self, order):
        """Parameters, moments and gradients as views of flat buffers in `order` (the order the
        backward finalises the gradients); one fused Adam over them, sharing the caller's lr
        tensor.  Same elementwise update as the caller's fused Adam, so the same bits."""
        opt = self.opt
        grp = opt.param_groups[0]
        used, seen = [], set()
        for p in order:  # gradient-ready order, each parameter once
            if id(p) not in seen and "exp_avg" in opt.state.get(p, {}):
                used.append(p)
                seen.add(id(p))
        missing = [p for p in self.params if id(p) not in seen and p.grad is not None]
        if missing:
            raise RuntimeError("GraphedStep: a parameter with a gradient has no Adam state")
        steps = [opt.state[p]["step"] for p in used]
        if not all(torch.equal(steps[0], st) for st in steps[1:]):
            raise RuntimeError("GraphedStep: the parameters' Adam step counters differ")
        dev = used[0].device
        if not torch.is_tensor(grp["lr"]):
            grp["lr"] = torch.tensor(float(grp["lr"]), device=dev)
        self._lr = grp["lr"]
        # every parameter view starts 16-byte aligned (4 floats; the padding stays 0): kernels
        # read weights with 16-byte vector loads, which a view at an arbitrary 4-byte offset
        # would break (the round-5 cost-volume forward read wrong W1 rows / faulted that way)
        al = lambda x: (x + 3) & ~3  # noqa: E731
        n = 0
        for p in used:
            n = al(n) + p.numel()
        P = torch.zeros(al(n), device=dev, dtype=used[0].dtype)
        M, V, G = torch.zeros_like(P), torch.zeros_like(P), torch.zeros_like(P)
        self._gviews, self._used, self._offs, off = [], used, [], 0
        with torch.no_grad():
            for p in used:
                off = al(off)
                k, st = p.numel(), opt.state[p]
                P[off:off + k].copy_(p.reshape(-1))
                M[off:off + k].copy_(st["exp_avg"].reshape(-1))
                V[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                p.data = P[off:off + k].view_as(p)
                st["exp_avg"] = M[off:off + k].view_as(p)  # the eager optimizer shares them
                st["exp_avg_sq"] = V[off:off + k].view_as(p)
                self._gviews.append(G[off:off + k].view_as(p))
                self._offs.append(off)
                off += k
        self.G = G
        # the per-parameter Adam step counters become views of one buffer: the tail keeps
        # them in sync with the flat optimizer's counter in one launch instead of a
        # foreach copy over ~240 scalars
        S = torch.empty(len(used), device=steps[0].device, dtype=steps[0].dtype)
        with torch.no_grad():
            S.copy_(torch.stack([st.reshape(()) for st in steps]))
        for i, p in enumerate(used):
            opt.state[p]["step"] = S[i].view_as(steps[i])
        self._steps = S
        flat = torch.nn.Parameter(P)
        flat.grad = G
        fo = torch.optim.Adam([flat], lr=self._lr, betas=grp["betas"], eps=grp["eps"],
                              weight_decay=grp["weight_decay"], maximize=grp["maximize"],
                              fused=True, capturable=True)
        fo.state[flat] = {"step": steps[0].clone(), "exp_avg": M, "exp_avg_sq": V}
        self.flat_opt = fo
        self._flat_step = fo.state[flat]["step"]
        # the update itself runs as one full-chip HIP launch (csrc/adam.hip) instead of
        # torch's multi-tensor fused Adam (7 launches of 40-57 workgroups over ~20 M floats:
        # 308 us per step); same elementwise arithmetic, same bits (tests/test_gpu_adam.py)
        if grp.get("amsgrad", False) or grp.get("differentiable", False):
            raise ValueError("GraphedStep: amsgrad / differentiable Adam is not supported")
        self._pmv = (P, M, V)
        self._adam_hp = (grp["betas"][0], grp["betas"][1], grp["eps"], grp["weight_decay"],
                         bool(grp["maximize"]))
        # gradient buckets (world > 1): consecutive runs of `used` of about bucket_bytes
        self.buckets = []
        if self.schedule == "overlap":
            cur, nb = [], 0
            for i, p in enumerate(used):
                cur.append(i)
                nb += p.numel() * p.element_size()
                if nb >= self.bucket_bytes or i == len(used) - 1:
                    lo = self._offs[cur[0]]
                    hi = self._offs[cur[-1]] + used[cur[-1]].numel()
                    self.buckets.append({"idx": cur, "lo": lo, "hi": hi, "left": len(cur),
                                         "done": False})
                    cur, nb = [], 0

    def _bucket_hooks(self):
        """Capture-time hooks: when the backward has finalised every gradient of a bucket,
        pack them into the bucket's slice of G (capture stream) and all-reduce that slice on
        the communication stream, forked from the capture stream at this point."""
        where = {}
        for bi, b in enumerate(self.buckets):
            b["left"], b["done"] = len(b["idx"]), False
            for i in b["idx"]:
                where[id(self._used[i])] = bi

        def hook(p):
            bi = where.get(id(p))
            if bi is None:
                return
            b = self.buckets[bi]
            b["left"] -= 1
            if b["left"] == 0:
                idx = b["idx"]
                # only this bucket's parameter gradients still in flight on their own stream
                wgrad.wait_for([self._used[i] for i in idx])
                _nat.copy_segments([self._gviews[i] for i in idx],
                                   [self._used[i].grad for i in idx])
                self.comm.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm):
                    dist.all_reduce(self.G[b["lo"]:b["hi"]])
                b["done"] = True
        return [p.register_post_accumulate_grad_hook(hook) for p in self._used]

    def _pack(self):
        _nat.copy_segments(self._gviews, [p.grad for p in self._used])

    def _tail(self, fork, pack=True):
        """Flat Adam step (+ the prefetched FPS handed over), inside a graph."""
        if pack:
            self._pack()
        # an eager optimizer step in between advanced the per-parameter counters
        self._flat_step.copy_(self._steps[0])
        if HIP_ADAM:
            self._flat_step.add_(1)  # as torch's fused Adam: the counter advances, then the update
            P, M, V = self._pmv
            _nat.adam_step(P, self.G, M, V, self._lr, self._flat_step, *self._adam_hp)
        else:
            self.flat_opt.step()
        self._steps.copy_(self._flat_step.reshape(1).expand_as(self._steps))
        if fork is not None:
            _nat.copy_segments(self.fps_cur, [t.contiguous() for t in self.fps_next])

    def _fps_kw(self, fps):
        return {} if self.prefetch_fn is None else {"fps": fps}

    def _eager_prefetch(self):
        if self.prefetch_fn is None:
            return None
        return list(self.prefetch_fn(*self.static[:self.n_prefetch]))

    @staticmethod
    def _key(ts):
        return tuple(ts), tuple(t._version for t in ts)

    def _allreduce_eager(self):
        """Warm-up path: the same averaging as the graphed step, eagerly (also initialises
        the communicator before any capture)."""
        if self.world == 1 and self.schedule != "overlap":
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        torch._foreach_div_(grads, float(self.world))

    def _sync_lr(self):
        """A plain `param_groups[0]['lr'] = x` replaced the shared tensor: fold it back."""
        grp = self.opt.param_groups[0]
        lr = grp["lr"]
        if lr is not self._lr:
            self._lr.fill_(float(lr))
            grp["lr"] = self._lr

    def __call__(self, *inputs, next_batch=None):
        self._sync_lr()
        for s, t in zip(self.static, inputs):
            s.copy_(t, non_blocking=True)
        if self.prefetch_fn is not None:
            cur = inputs[:self.n_prefetch]
            hit = False
            if self._pending is not None:
                ts, ver = self._pending
                hit = (len(ts) == len(cur) and all(a is b for a, b in zip(ts, cur))
                       and ver == tuple(t._version for t in cur))
            if not hit:  # not prefetched by the previous replay: compute it now
                torch._foreach_copy_(self.fps_cur, self._eager_prefetch())
            nxt = inputs if next_batch is None else next_batch
            for s, t in zip(self.static_next, nxt[:self.n_prefetch]):
                s.copy_(t, non_blocking=True)
            self._pending = (self._key(nxt[:self.n_prefetch]) if next_batch is not None
                             else None)
        self._replay()
        if self.graph_b is not None:
            dist.all_reduce(self.G)
            self.graph_b.replay()
        return self.loss.detach()


def graphed_flow_step(model, optimizer, example_inputs, loss_fn=None, warmup=3, prefetch=True,
                      overlap=None):
    """FlowTrainStep as a GraphedStep (model: the bare module, not DDP-wrapped).  prefetch:
    the next batch's FPS chain runs inside graph A on a forked stream (see GraphedStep)."""
    loss_fn = loss_fn or loss_functions.multiScaleLoss
    model.train()

    def run(pos1, pos2, flow, fps=None):
        kw = {} if fps is None else {"fps_idx": fps}
        flows, fps1, _, _, _, _, _, _ = model(pos1, pos2, pos1, pos2, **kw)
        return loss_fn(flows, flow, fps1)
    return GraphedStep(run, model.parameters(), optimizer, example_inputs, warmup,
                       prefetch_fn=_plan_fn(model) if prefetch else None, overlap=overlap)


def graphed_kd_step(teacher, student, optimizer, example_inputs, gamma=0.3, beta=0.8, layer=3,
                    warmup=3, prefetch=True, overlap=None):
    """KDTrainStep (distilTrain.py:164-182) as a GraphedStep; teacher and student share the
    (prefetched) FPS chain, as KDTrainStep does."""
    for p in teacher.parameters():
        p.requires_grad_(False)
    teacher.eval()
    student.train()

    def loss_from(s_out, t_out, pos1, pos2, flow):
        flows, fps1, fps2, _, _, feat1s, feat2s, _ = s_out
        t_flows, t_fps1, t_fps2, _, _, t_feat1s, t_feat2s, _ = t_out
        return loss_functions.biDirection_loss_ht(
            flows, feat1s, feat2s, fps1, fps2, flow, t_flows, t_feat1s, t_feat2s, t_fps1, t_fps2,
            gamma, beta, layer=layer)

    def teacher_fwd(pos1, pos2, flow, fps=None):
        kw = {} if fps is None else {"fps_idx": fps}
        with torch.no_grad():
            return teacher(pos1, pos2, pos1, pos2, **kw)

    def student_fwd(pos1, pos2, flow, fps=None):
        kw = {} if fps is None else {"fps_idx": fps}
        with _kd_student_streams(student):
            return student(pos1, pos2, pos1, pos2, **kw)

    def run(pos1, pos2, flow, fps=None):  # the eager form (warm-up; TEACHER_GRAPH = False)
        kw = {} if fps is None else {"fps_idx": fps}
        t_fork = _TeacherFork(teacher, (pos1, pos2, pos1, pos2), kw)
        s_out = student_fwd(pos1, pos2, flow, fps)
        return loss_from(s_out, t_fork.join(), pos1, pos2, flow)
    stages = (teacher_fwd, student_fwd, loss_from) if TEACHER_GRAPH else None
    return GraphedStep(run, student.parameters(), optimizer, example_inputs, warmup,
                       prefetch_fn=_plan_fn(student) if prefetch else None, overlap=overlap,
                       stages=stages)
