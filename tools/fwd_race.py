"""Self-consistency of captured FORWARD passes run on two streams (KD teacher race).

A HIP graph holds one or two model forwards (the KD step's frozen teacher and/or the student),
each on a chosen stream, with fixed inputs; it is replayed R times and every replay's outputs
are compared with the first replay's.  Any difference is a race (same kernels, same inputs).

  python tools/fwd_race.py VARIANT [reps=200] [plan=1] [b=4] [n=8192]
VARIANT (side stream | capture stream):
  ts        teacher no_grad | student grad       (the KD step's forward)
  t_side    teacher no_grad | -                  (teacher alone on a forked stream)
  t_inline  -               | teacher no_grad
  tt        teacher no_grad | teacher copy no_grad
  tg_s      teacher grad-mode (frozen) | student grad
  s_side    student grad    | teacher no_grad    (streams swapped)
  ss        student grad    | student copy grad
ops=1: every op the side-stream model issues has its outputs cloned into the graph (a
dispatch mode active during the capture), and a mismatching replay names the first op, in
issue order, whose output differs from the first replay's.
"""
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kd-pointcloud_amd"))
import torch  # noqa: E402

DEV = "cuda"


def main():
    var = sys.argv[1]
    o = dict(a.split("=") for a in sys.argv[2:])
    reps, b, n = int(o.get("reps", 200)), int(o.get("b", 4)), int(o.get("n", 8192))
    use_plan = o.get("plan", "1") == "1"
    import synthetic
    import kdpc_native
    import pointconv_util as PU
    # off=pc,cv,wn,ws,idw,tile,bn: replace fused HIP kernels by their torch formulations
    # (the test seams), to bisect which kernel the race needs
    seams = {"pc": (PU, "_FUSED_POINTCONV"), "cv": (PU, "_FUSED_COST_VOLUME"),
             "wn": (PU, "_FUSED_WEIGHTNET"), "ws": (PU, "_FUSED_WSUM"), "idw": (PU, "_FUSED_IDW"),
             "bn": (PU, "_FUSED_BN"), "tile": (kdpc_native, "TILED_FWD")}
    for k in [x for x in o.get("off", "").split(",") if x]:
        setattr(*seams[k], False)
    print("off:", o.get("off", ""), flush=True)
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    torch.manual_seed(1)
    teacher = Teacher().to(DEV).eval()
    for p in teacher.parameters():
        p.requires_grad_(False)
    torch.manual_seed(2)
    student = Student().to(DEV).train()
    p1, p2, _ = (torch.from_numpy(a).to(DEV) for a in synthetic.ft3d_batch(b, n, seed=31))
    plan = [t.clone() for t in student.precompute_plan(p1, p2)] if use_plan else None
    models = {"t": teacher, "t2": copy.deepcopy(teacher), "s": student,
              "s2": copy.deepcopy(student)}
    # (side, main) -> (model key, grad enabled)
    spec = {"ts": (("t", False), ("s", True)), "t_side": (("t", False), None),
            "t_inline": (None, ("t", False)), "tt": (("t", False), ("t2", False)),
            "tg_s": (("t", True), ("s", True)), "s_side": (("s", True), ("t", False)),
            "ss": (("s", True), ("s2", True))}[var]
    side = torch.cuda.Stream()
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch.utils._pytree import tree_flatten

    class OpStash(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.rec = []

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func)
            if window[0] and name.startswith("kdpc."):  # a HIP op's inputs, as it reads them
                for i, t in enumerate(tree_flatten((args, kwargs))[0]):
                    if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() > 0:
                        self.rec.append((f"{len(self.rec)}:{name}:in{i}", t.detach().clone()))
            out = func(*args, **(kwargs or {}))
            skip = ("record_stream", "empty", "view", "aten.t.", "slice", "split", "reshape",
                    "expand", "permute", "select", "squeeze", "detach", "alias", "as_strided",
                    "transpose")
            if not any(k in name for k in skip) and window[0]:
                for i, t in enumerate(tree_flatten(out)[0]):
                    if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() > 0:
                        self.rec.append((f"{len(self.rec)}:{name}[{i}]", t.detach().clone()))
            return out

    # win=i: with pcstash=1, also every op between the side model's PointConv calls i and i+1
    win = int(o.get("win", -1))
    window = [win < 0]
    stash = OpStash() if o.get("ops", "0") == "1" or win >= 0 else None
    capturing = [False]
    # pcstash=1: only the fused PointConv forwards of the side-stream model (inputs and
    # output) are cloned into the graph -- little extra work, so the race stays visible
    pc_rec = []
    if o.get("pcstash", "0") == "1":
        stash = stash if win >= 0 else None
        orig = {n_: getattr(kdpc_native, n_) for n_ in ("pointconv_fwd", "pointconv_fwd_tiled")}

        def wrap(n_):
            def f(*a):
                on_side = capturing[0] and torch.cuda.current_stream() == side
                if on_side and win >= 0:
                    window[0] = False
                y = orig[n_](*a)
                if on_side:
                    i = len(pc_rec) // 6
                    if win >= 0:
                        window[0] = i == win
                    xyz, center, feats, idx, wt = a[:5]
                    tag = f"pc{i}:{n_}:S={idx.shape[1]},K={idx.shape[2]},D={feats.shape[2]}," \
                          f"O={a[5].shape[0]}"
                    for nm, t in (("xyz", xyz), ("feats", feats), ("idx", idx), ("wt", wt),
                                  ("wl", a[5]), ("y", y)):
                        pc_rec.append((f"{tag}:{nm}", t.detach().clone()))
                return y
            return f
        for n_ in orig:
            setattr(kdpc_native, n_, wrap(n_))

    def fwd(which, is_side=False):
        key, grad = which
        kw = {} if plan is None else {"fps_idx": plan}
        with torch.set_grad_enabled(grad):
            if is_side and stash is not None and capturing[0]:
                with stash:
                    out = models[key](p1, p2, p1, p2, **kw)
            else:
                out = models[key](p1, p2, p1, p2, **kw)
        return [t.detach().clone() for t in out[0]] + [out[5][3].detach().clone()]

    def body():
        cur = torch.cuda.current_stream()
        res = {}
        if spec[0] is not None:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                res["side"] = fwd(spec[0], True)
        if spec[1] is not None:
            res["main"] = fwd(spec[1])
        if spec[0] is not None:
            cur.wait_stream(side)
        return res

    # warm-up (lazy state) eagerly, then capture
    body()
    torch.cuda.synchronize()
    if o.get("memhist", "0") == "1":
        torch.cuda.memory._record_memory_history(max_entries=1000000)
    two = o.get("graphs", "1") == "2"
    g = torch.cuda.CUDAGraph()
    capturing[0] = True
    if not two:
        with torch.cuda.graph(g):
            outs = body()
    else:
        # one graph per stream: the side model's forward captured on the side stream, the main
        # one's on the capture stream; replayed concurrently, joined by ordinary stream events
        g_side = torch.cuda.CUDAGraph()
        outs = {}
        with torch.cuda.graph(g_side, stream=side):
            outs["side"] = fwd(spec[0], True)
        with torch.cuda.graph(g):
            outs["main"] = fwd(spec[1])

        g_main = g

        class _Two:
            def replay(self):
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    g_side.replay()
                g_main.replay()
                cur.wait_stream(side)
        two_obj = _Two()
    capturing[0] = False
    torch.cuda.synchronize()
    if o.get("memhist", "0") == "1":
        snap = torch.cuda.memory._snapshot()
        torch.cuda.memory._record_memory_history(enabled=None)
        ev = [e for tr in snap["device_traces"] for e in tr]
        allocs = [(e["addr"], e["addr"] + e["size"], e["stream"]) for e in ev
                  if e["action"] == "alloc"]
        streams = sorted({a[2] for a in allocs})
        print(f"memhist: {len(ev)} events, {len(allocs)} allocs in the capture, streams {streams}",
              flush=True)
        by_stream = {st: sorted((a, b) for a, b, s2 in allocs if s2 == st) for st in streams}
        # any address range handed to two streams?
        import bisect
        hits = []
        for i, sa in enumerate(streams):
            for sb in streams[i + 1:]:
                lst = by_stream[sb]
                starts = [x[0] for x in lst]
                for a, b in by_stream[sa]:
                    j = bisect.bisect_right(starts, b - 1)
                    for k in range(max(0, j - 64), j):
                        c, d = lst[k]
                        if c < b and a < d:
                            hits.append((sa, hex(a), b - a, sb, hex(c), d - c))
        print(f"memhist: address ranges allocated on two different streams: {len(hits)}; "
              f"first: {hits[:10]}", flush=True)
        segs = snap["segments"]
        print("memhist: segments by stream:",
              {st: sum(1 for sg in segs if sg["stream"] == st) for st in {sg["stream"] for sg in segs}},
              flush=True)
    g.replay()
    torch.cuda.synchronize()
    ref = {k: [t.clone() for t in v] for k, v in outs.items()}
    sref = [t.clone() for _, t in stash.rec] if stash is not None else []
    pref = [t.clone() for _, t in pc_rec]
    first_ops = {}
    first_win = {}
    bad = {k: 0 for k in outs}
    worst = {k: 0.0 for k in outs}
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    print(f"replay ms (20 back to back): {(time.perf_counter() - t0) / 20 * 1e3:.3f}", flush=True)
    for r in range(reps):
        g.replay()
        if r % 10 == 9 or r == reps - 1:
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        for k, v in outs.items():
            d = [float((a - c).abs().max() / (c.abs().max() + 1e-30))
                 for a, c in zip(v, ref[k]) if not torch.equal(a, c)]
            if d:
                bad[k] += 1
                worst[k] = max(worst[k], max(d))
        if stash is not None:
            for (nm, t), t0 in zip(stash.rec, sref):
                if not torch.equal(t, t0):
                    first_win[nm] = first_win.get(nm, 0) + 1
                    break
        if pc_rec:
            diffs = [nm for (nm, t), t0 in zip(pc_rec, pref) if not torch.equal(t, t0)]
            if diffs:
                key = " | ".join(diffs[:3])
                first_ops[key] = first_ops.get(key, 0) + 1
        if r % 50 == 49:
            print(f"  {r + 1} replays: mismatching replays {bad}", flush=True)
    print(f"RESULT {var} plan={int(use_plan)} reps={reps} mismatching replays {bad} "
          f"worst rel {worst}", flush=True)
    if pc_rec:
        print(f"side PointConv tensors stashed: {len(pc_rec)}; first differing per replay:",
              flush=True)
        for kk, v in sorted(first_ops.items(), key=lambda kv: -kv[1]):
            print(f"   {v:4d} x {kk}", flush=True)
    if stash is not None:
        print(f"side ops stashed: {len(stash.rec)}; first differing op per replay: "
              f"{sorted(first_win.items(), key=lambda kv: int(kv[0].split(':')[0]))}", flush=True)
        for nm, _ in stash.rec:
            print("   op", nm, flush=True)


if __name__ == "__main__":
    main()
