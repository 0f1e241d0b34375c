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
import torch
import torch.distributed as dist

import kdpc_native
import loss_functions


def is_dist():
    return dist.is_available() and dist.is_initialized()


def wrap_ddp(model, device=None):
    """Wrap the trained model for DDP when a process group is up (no-op otherwise)."""
    if not is_dist() or dist.get_world_size() == 1:
        return model
    kw = dict(broadcast_buffers=True, static_graph=True, gradient_as_bucket_view=True)
    if device is not None and device.type == "cuda":
        kw["device_ids"] = [device.index]
    return torch.nn.parallel.DistributedDataParallel(model, **kw)


def make_optimizer(model, lr=1e-3, weight_decay=1e-4, capturable=False):
    """Adam as configured by config_train_kd_pointconv.yaml:15-24 / distilTrain.py:134-135.
    capturable=True keeps the step counters on the device (required by GraphedStep).  On
    the GPU the fused (single multi-tensor kernel) implementation is used: the same Adam
    update (L2 weight decay, not AdamW) in one launch instead of ~10 foreach passes."""
    params = list(model.parameters())
    fused = len(params) > 0 and all(p.is_cuda for p in params)
    return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-08,
                            weight_decay=weight_decay, capturable=capturable,
                            fused=True if fused else None)


def _core(model):
    return model.module if isinstance(model, torch.nn.parallel.DistributedDataParallel) else model


class FpsPrefetch:
    """Runs the encoder's FPS chain (PointConvBidirection.precompute_fps) for an upcoming
    batch on a side HIP stream.  FPS is one workgroup per cloud for ~2900 dependent steps
    (2.5 ms per B=8 step, latency-bound on 16 CUs); issued one step ahead it runs beside the
    current step's kernels instead of in front of them.  Results are identical to computing
    FPS inside the forward (same kernel, same inputs)."""

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
            self.fps = _core(model).precompute_fps(pos1, pos2)
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
            fps = _core(self.student).precompute_fps(pos1, pos2)
        if next_batch is not None:
            self.prefetch.launch(self.student, next_batch[0], next_batch[1])
        kw = {} if fps is None else {"fps_idx": fps}
        self.teacher.eval()
        with torch.no_grad():
            t_flows, t_fps1, t_fps2, _, _, t_feat1s, t_feat2s, _ = self.teacher(
                pos1, pos2, color1, color2, **kw)
        self.student.train()
        flows, fps1, fps2, _, _, feat1s, feat2s, _ = self.student(pos1, pos2, color1, color2,
                                                                  **kw)
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


class GraphedStep:
    """One training step replayed from HIP graphs (MI355X: the eager step issues ~2000
    launches per iteration from Python, ~21 ms of host time, about as much as the GPU needs).

        graph A: [FPS of the NEXT batch on a forked stream] + forward + loss + backward
                 (+ packing the gradients into one flat buffer)
        eager:   one all_reduce of the flat gradient buffer (world > 1; RCCL over xGMI)
        graph B: unpack the averaged gradients + optimizer step (Adam, capturable=True)
    With one process there is no all-reduce and the optimizer step is captured at the end of
    graph A (a single graph per step).

    The collective stays outside the graphs on purpose: it is one 31.8 MB all-reduce per
    step, and keeping it eager avoids depending on collective capture.  `loss_fn(*inputs)`
    must run the whole forward (model call(s) and loss) and return the loss; the inputs are
    copied into static buffers before each replay.  Warm-up iterations run eagerly on a side
    stream (they allocate lazily-initialised state: optimizer moments, cached attributes).

    prefetch_fn (optional, e.g. PointConvBidirection.precompute_fps): a function of the first
    `n_prefetch` inputs whose result loss_fn takes as `fps=`.  Graph A then runs it for the
    next batch on a forked stream, beside this batch's forward/backward (FpsPrefetch inside
    the graph: FPS is ~2.4 ms of latency-bound work on 16 CUs), into buffers the next replay
    reads.  A call whose batch is not the previous call's `next_batch` recomputes it eagerly
    first, so results never depend on what was prefetched."""

    drop_warmup_graph = True  # diagnostics seam (tools/graph_diag.py)
    flat_adam = True  # seam: False keeps the caller's per-tensor optimizer step
    capture_on_side_stream = False

    def __init__(self, loss_fn, params, optimizer, example_inputs, warmup=3, prefetch_fn=None,
                 n_prefetch=2):
        self.loss_fn = loss_fn
        self.opt = optimizer
        self.params = [p for p in params if p.requires_grad]
        self.static = [t.detach().clone() for t in example_inputs]
        self.world = dist.get_world_size() if is_dist() else 1
        self.prefetch_fn = prefetch_fn
        self.n_prefetch = n_prefetch
        self.static_next = [t.detach().clone() for t in example_inputs[:n_prefetch]]
        self._pending = None  # (tensors, versions) the buffered prefetch was computed for
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loss = None
            for _ in range(warmup):
                self.opt.zero_grad(set_to_none=True)
                loss = self.loss_fn(*self.static, **self._fps_kw(self._eager_prefetch()))
                loss.backward()
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
        self.flat_opt = self._flat_adam() if self.world == 1 and self.flat_adam else None
        # graph A: forward + backward; .grad tensors are allocated inside (static addresses)
        self.opt.zero_grad(set_to_none=True)
        self.graph_a = torch.cuda.CUDAGraph()
        kw = {"stream": side} if self.capture_on_side_stream else {}
        if self.world > 1:
            # a process group's background threads (RCCL watchdog: event queries) may touch the
            # runtime while this thread captures; "global" mode would fail those calls
            kw["capture_error_mode"] = "thread_local"
        fork = torch.cuda.Stream() if prefetch_fn is not None else None
        with torch.cuda.graph(self.graph_a, **kw):
            cap = torch.cuda.current_stream()
            if fork is not None:
                # graph B of the previous replay copied its fps_next into fps_cur
                fork.wait_stream(cap)
                with torch.cuda.stream(fork):
                    self.fps_next = list(prefetch_fn(*self.static_next))
            self.loss = self.loss_fn(*self.static, **self._fps_kw(self.fps_cur))
            self.loss.backward()
            kdpc_native.csr_join()  # side-stream CSR builds (csr_prefetch) rejoin the capture
            self.grads = [p.grad for p in self.params if p.grad is not None]
            self.flat = torch.cat([g.reshape(-1) for g in self.grads]) if self.world > 1 else None
            if fork is not None:
                cap.wait_stream(fork)
            if self.world == 1:  # nothing runs between the halves: one graph, one launch
                self._tail(fork)
        # graph B: unpack + optimizer step (+ hand the prefetched FPS to the next replay);
        # a second graph launch costs ~0.5 ms of idle GPU between the replays (rocprofv3,
        # round 2), so it exists only when the all-reduce has to run between the two
        self.graph_b = None
        if self.world > 1:
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b, pool=self.graph_a.pool(), **kw):
                self._unpack()
                self._tail(fork)
        torch.cuda.synchronize()
        # keep the static loss buffer, not the captured autograd graph: while that graph
        # lives, an eager step on the same parameters reuses its AccumulateGrad nodes (bound
        # to the capture stream) and torch warns of a stream mismatch (bench's eager
        # measurement steps after the timed region)
        self.loss = self.loss.detach()
        self._pending = None

    def _flat_adam(self):
        """One flat Adam over the trained parameters instead of the per-tensor fused Adam: the
        parameters (and the optimizer's moments) become views of flat buffers, the step copies
        the ~440 gradient tensors into one buffer and updates all 8 M values in one pass (the
        per-tensor fused Adam: 7 launches, ~0.3 ms for 31.8 MB).  Same elementwise update, so
        the same bits.  Only for a single-group fused capturable Adam; None otherwise."""
        opt = self.opt
        if type(opt) is not torch.optim.Adam or len(opt.param_groups) != 1:
            return None
        grp = opt.param_groups[0]
        if not grp.get("fused") or not grp.get("capturable") or grp.get("amsgrad"):
            return None
        used = [p for p in grp["params"] if "exp_avg" in opt.state.get(p, {})]
        if not used:
            return None
        steps = [opt.state[p]["step"] for p in used]
        if not all(torch.equal(steps[0], st) for st in steps[1:]):
            return None
        n = sum(p.numel() for p in used)
        P = torch.empty(n, device=used[0].device, dtype=used[0].dtype)
        M, V, G = torch.empty_like(P), torch.empty_like(P), torch.zeros_like(P)
        self._gviews, self._used, off = [], used, 0
        with torch.no_grad():
            for p in used:
                k, st = p.numel(), opt.state[p]
                P[off:off + k].copy_(p.reshape(-1))
                M[off:off + k].copy_(st["exp_avg"].reshape(-1))
                V[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                p.data = P[off:off + k].view_as(p)
                st["exp_avg"] = M[off:off + k].view_as(p)  # the eager optimizer shares them
                st["exp_avg_sq"] = V[off:off + k].view_as(p)
                self._gviews.append(G[off:off + k].view_as(p))
                off += k
        flat = torch.nn.Parameter(P)
        flat.grad = G
        fo = torch.optim.Adam([flat], lr=grp["lr"], betas=grp["betas"], eps=grp["eps"],
                              weight_decay=grp["weight_decay"], maximize=grp["maximize"],
                              fused=True, capturable=True)
        fo.state[flat] = {"step": steps[0].clone(), "exp_avg": M, "exp_avg_sq": V}
        return fo

    def _tail(self, fork):
        if self.flat_opt is not None:
            torch._foreach_copy_(self._gviews, [p.grad for p in self._used])
            self.flat_opt.step()
        else:
            self.opt.step()
        if fork is not None:
            for c, n in zip(self.fps_cur, self.fps_next):
                c.copy_(n)

    def _fps_kw(self, fps):
        return {} if self.prefetch_fn is None else {"fps": fps}

    def _eager_prefetch(self):
        if self.prefetch_fn is None:
            return None
        return list(self.prefetch_fn(*self.static[:self.n_prefetch]))

    @staticmethod
    def _key(ts):
        return tuple(ts), tuple(t._version for t in ts)

    def _unpack(self):
        off = 0
        for g in self.grads:
            n = g.numel()
            g.copy_(self.flat[off:off + n].view_as(g))
            off += n
        torch._foreach_div_(self.grads, float(self.world))

    def _allreduce_eager(self):
        """Warm-up path: the same averaging as the graphed step, eagerly."""
        if self.world == 1:
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        torch._foreach_div_(grads, float(self.world))

    def __call__(self, *inputs, next_batch=None):
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
                for c, n in zip(self.fps_cur, self._eager_prefetch()):
                    c.copy_(n)
            nxt = inputs if next_batch is None else next_batch
            for s, t in zip(self.static_next, nxt[:self.n_prefetch]):
                s.copy_(t, non_blocking=True)
            self._pending = (self._key(nxt[:self.n_prefetch]) if next_batch is not None
                             else None)
        self.graph_a.replay()
        if self.graph_b is not None:
            dist.all_reduce(self.flat)
            self.graph_b.replay()
        return self.loss.detach()


def graphed_flow_step(model, optimizer, example_inputs, loss_fn=None, warmup=3, prefetch=True):
    """FlowTrainStep as a GraphedStep (model: the bare module, not DDP-wrapped).  prefetch:
    the next batch's FPS chain runs inside graph A on a forked stream (see GraphedStep)."""
    loss_fn = loss_fn or loss_functions.multiScaleLoss
    model.train()

    def run(pos1, pos2, flow, fps=None):
        kw = {} if fps is None else {"fps_idx": fps}
        flows, fps1, _, _, _, _, _, _ = model(pos1, pos2, pos1, pos2, **kw)
        return loss_fn(flows, flow, fps1)
    return GraphedStep(run, model.parameters(), optimizer, example_inputs, warmup,
                       prefetch_fn=model.precompute_fps if prefetch else None)


def graphed_kd_step(teacher, student, optimizer, example_inputs, gamma=0.3, beta=0.8, layer=3,
                    warmup=3, prefetch=True):
    """KDTrainStep (distilTrain.py:164-182) as a GraphedStep; teacher and student share the
    (prefetched) FPS chain, as KDTrainStep does."""
    for p in teacher.parameters():
        p.requires_grad_(False)
    teacher.eval()
    student.train()

    def run(pos1, pos2, flow, fps=None):
        kw = {} if fps is None else {"fps_idx": fps}
        with torch.no_grad():
            t_flows, t_fps1, t_fps2, _, _, t_feat1s, t_feat2s, _ = teacher(pos1, pos2, pos1, pos2,
                                                                           **kw)
        flows, fps1, fps2, _, _, feat1s, feat2s, _ = student(pos1, pos2, pos1, pos2, **kw)
        return loss_functions.biDirection_loss_ht(
            flows, feat1s, feat2s, fps1, fps2, flow, t_flows, t_feat1s, t_feat2s, t_fps1, t_fps2,
            gamma, beta, layer=layer)
    return GraphedStep(run, student.parameters(), optimizer, example_inputs, warmup,
                       prefetch_fn=student.precompute_fps if prefetch else None)
