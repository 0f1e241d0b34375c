"""kNN (csrc/knn.hip) under concurrency: two streams of one HIP graph each run a chain of
knn_point calls of the models' shapes; the graph is replayed R times and every result is
compared with the first replay's (tools/fwd_race.py localised the KD teacher race to the
level-2 cost volume's kNN, the plain scan knn_kernel<4> at N=512).

  python tools/knn_race.py [main=knn|gemm|none] [reps=300] [shapes=all|small|model]
shapes=model: the inputs of every knn_point call of one eager teacher forward (B=4, N=8192,
with the coordinate plan), recorded and replayed as they were.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kd-pointcloud_amd"))
import torch  # noqa: E402

DEV = "cuda"
# (clouds, refs N, queries S, K): cost volumes (K=32), warping / upsampling 3-NN, estimators
SHAPES = {"all": [(8, 512, 512, 32), (8, 256, 256, 32), (8, 2048, 2048, 32), (16, 8192, 8192, 32),
                  (4, 512, 2048, 3), (4, 2048, 8192, 3), (4, 512, 512, 9), (4, 2048, 2048, 9)],
          "small": [(8, 512, 512, 32), (8, 256, 256, 32), (4, 512, 512, 9)]}


def main():
    o = dict(a.split("=") for a in sys.argv[1:])
    reps, main_kind = int(o.get("reps", 300)), o.get("main", "knn")
    import kdpc_native as K
    shapes = SHAPES.get(o.get("shapes", "all"))
    g = torch.Generator(device="cpu").manual_seed(0)

    def inputs():
        return [(torch.rand(b, n, 3, generator=g).to(DEV), torch.rand(b, s, 3, generator=g).to(DEV),
                 k) for b, n, s, k in shapes]
    if o.get("shapes") == "model":
        import synthetic
        from models_bid_pointconv import PointConvBidirection as Teacher
        torch.manual_seed(1)
        teacher = Teacher().to(DEV).eval()
        p1, p2, _ = (torch.from_numpy(a).to(DEV) for a in synthetic.ft3d_batch(4, 8192, seed=31))
        plan = teacher.precompute_plan(p1, p2)
        rec = []
        orig = K.knn_point

        def spy(nsample, xyz, new_xyz, *a, **kw):
            rec.append((xyz.detach().clone(), new_xyz.detach().clone(), nsample))
            return orig(nsample, xyz, new_xyz, *a, **kw)
        K.knn_point = spy
        with torch.no_grad():
            teacher(p1, p2, p1, p2, fps_idx=plan)
        K.knn_point = orig
        shapes = [(x.shape[0], x.shape[1], q.shape[1], k) for x, q, k in rec]
        print("model knn calls:", shapes, flush=True)
        ins = {"side": rec, "main": [(x.clone(), q.clone(), k) for x, q, k in rec]}
        import copy
        t_main = copy.deepcopy(teacher)
    else:
        ins = {"side": inputs(), "main": inputs()}
    gemm = [(torch.randn(16384, 256, generator=g).to(DEV), torch.randn(256, 256, generator=g).to(DEV))
            for _ in range(6)]

    twice = o.get("twice", "0") == "1"
    wsmode = o.get("ws", "")  # same | fresh: explicit workspaces through the C ABI (culled calls)
    if wsmode:
        lib = K.load_library()
        wss = {}
        for key in ("side",):
            for j, (x, q, k) in enumerate(ins[key]):
                nb = lib.kdpc_knn_workspace_bytes(x.shape[0], x.shape[1], q.shape[1])
                if nb:
                    wss[(key, j)] = [torch.empty(nb, dtype=torch.uint8, device=DEV)
                                     for _ in range(2)]

    def knn_ws(k, x, q, ws):
        idx = torch.empty((x.shape[0], q.shape[1], k), dtype=torch.int32, device=DEV)
        rc = lib.kdpc_knn_point_ws(x.shape[0], x.shape[1], q.shape[1], k, x.data_ptr(),
                                   q.data_ptr(), idx.data_ptr(), None, ws.data_ptr(),
                                   ws.numel(), torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        return idx

    def knn_chain(key):
        if not twice:
            return [K.knn_point(k, x, q) for x, q, k in ins[key]]
        # each search twice in a row on the same inputs, and the inputs checksummed after them
        # (a difference between the two results is the kernel's own; a changed input is not)
        out = []
        for j, (x, q, k) in enumerate(ins[key]):
            w = wss.get((key, j)) if wsmode else None
            if w is not None:
                out += [knn_ws(k, x, q, w[0]), knn_ws(k, x, q, w[0] if wsmode == "same" else w[1]),
                        x.clone(), q.clone()]
            else:
                out += [K.knn_point(k, x, q), K.knn_point(k, x, q), x.clone(), q.clone()]
        return out

    side = torch.cuda.Stream()

    def body():
        cur = torch.cuda.current_stream()
        res = {}
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            res["side"] = knn_chain("side")
        if main_kind == "knn":
            res["main"] = knn_chain("main")
        elif main_kind == "gemm":
            res["main"] = [a @ b for a, b in gemm]
        elif main_kind == "teacher":  # a whole model forward beside the kNN chain
            with torch.no_grad():
                res["main"] = list(t_main(p1, p2, p1, p2, fps_idx=plan)[0])
        cur.wait_stream(side)
        return res

    body()
    torch.cuda.synchronize()
    if o.get("eager", "0") == "1":  # no graph: the same two streams, launched eagerly
        class _Eager:
            def replay(self):
                res = body()
                for kk, v in res.items():
                    for dst, src in zip(outs[kk], v):
                        dst.copy_(src)
        outs = body()
        gr = _Eager()
    else:
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            outs = body()
    gr.replay()
    torch.cuda.synchronize()
    ref = {k: [t.clone() for t in v] for k, v in outs.items()}
    eager = knn_chain("side")
    torch.cuda.synchronize()
    vs_eager = [i for i, (a, c) in enumerate(zip(ref["side"], eager)) if not torch.equal(a, c)]
    if twice:  # within the first replay: run 1 vs run 2 of each call
        print("twice, first replay: run1 != run2 at calls",
              [j for j in range(len(ins["side"])) if not torch.equal(ref["side"][4 * j],
                                                                      ref["side"][4 * j + 1])],
              flush=True)
    bad = {k: 0 for k in outs}
    which = {}
    for r in range(reps):
        gr.replay()
        torch.cuda.synchronize()
        for k in outs:
            d = [i for i, (a, c) in enumerate(zip(outs[k], ref[k])) if not torch.equal(a, c)]
            if d:
                bad[k] += 1
                if k == "side" and bad[k] <= 4:
                    for i in [i for i in d if not twice or i % 4 < 2][:2]:
                        a, c = outs[k][i], ref[k][i]
                        rows = (a != c).any(-1).nonzero()
                        x, q, kk = ins[k][i // 4 if twice else i]
                        b0, s0 = (int(v) for v in rows[0])
                        def dd(ix):  # distances of in-range indices only (garbage -> nan)
                            ok = (ix >= 0) & (ix < x.shape[1])
                            v = ((x[b0, ix.clamp(0, x.shape[1] - 1).long()] - q[b0, s0]) ** 2
                                 ).sum(-1)
                            return torch.where(ok, v, torch.full_like(v, float("nan")))
                        print(f"  replay {r} call {i} {tuple(a.shape)}: {len(rows)} query rows "
                              f"differ (of {a.shape[0] * a.shape[1]}); first (b={b0}, q={s0}):\n"
                              f"    ref {c[b0, s0].tolist()}\n    got {a[b0, s0].tolist()}\n"
                              f"    ref d {[round(v, 6) for v in dd(c[b0, s0]).tolist()]}\n"
                              f"    got d {[round(v, 6) for v in dd(a[b0, s0]).tolist()]}",
                              flush=True)
                        # every differing row: is the result still a valid K-nearest set (same
                        # sorted distances as the reference row: a tie order difference) or not
                        da = ((x[rows[:, 0, None], a[rows[:, 0], rows[:, 1]].clamp(0, x.shape[1] - 1).long()]
                               - q[rows[:, 0], rows[:, 1]][:, None]) ** 2).sum(-1)
                        dc = ((x[rows[:, 0, None], c[rows[:, 0], rows[:, 1]].clamp(0, x.shape[1] - 1).long()]
                               - q[rows[:, 0], rows[:, 1]][:, None]) ** 2).sum(-1)
                        oor = int(((a[rows[:, 0], rows[:, 1]] < 0) | (a[rows[:, 0], rows[:, 1]] >= x.shape[1])).sum())
                        same_d = int((da.sort(-1)[0] == dc.sort(-1)[0]).all(-1).sum())
                        print(f"    rows differing {len(rows)}: same sorted distances {same_d}, "
                              f"out-of-range indices {oor}, rows per cloud "
                              f"{torch.bincount(rows[:, 0], minlength=a.shape[0]).tolist()}, "
                              f"query rows {rows[:8, 1].tolist()}", flush=True)
                for i in d:
                    key = (k, i) if twice else (k, shapes[i] if k == "side" or main_kind == "knn"
                                                else i)
                    which[key] = which.get(key, 0) + 1
    if twice:
        nc = len(ins["side"])
        intra = sum(v for (kk, i), v in which.items() if kk == "side")
        print(f"twice: per side output index mismatch counts (4 per call: run1, run2, xyz, "
              f"new_xyz) {sorted(((i, v) for (kk, i), v in which.items() if kk == 'side'))}",
              flush=True)
    if o.get("dbg") == "1":  # tools/variants/knn_dbg.py findings
        import ctypes
        import struct
        lib_d = ctypes.CDLL(K.LIB_PATH)
        buf = (ctypes.c_ulonglong * (8 + 64 * 8))()
        torch.cuda.synchronize()
        assert lib_d.kdpc_knn_dbg_read(buf, 0) == 0
        names = ["query record mismatch", "ref vs xyz mismatch", "ref outside its box",
                 "query short of K", "bad boxes (failing clouds)", "culled launches"]
        print("DBG", {nm: int(buf[i]) for i, nm in enumerate(names)}, flush=True)

        def f32(u):
            return struct.unpack("f", struct.pack("I", u & 0xffffffff))[0]
        for r in range(min(int(buf[7]), 64)):
            t, a, b2, c, d, e = (int(v) for v in buf[8 + r * 8: 8 + r * 8 + 6])
            if t == 3:
                print(f"  short: cloud {a >> 32} pos {a & 0xffffffff} cnt {b2} refs under final "
                      f"thr {c >> 32} under seed {c & 0xffffffff} seed {f32(d >> 32):.6g} final "
                      f"thr {f32(d):.6g} bad boxes {e}", flush=True)
            else:
                print(f"  {names[t]}: {a} {b2} {c} {d}", flush=True)
    print(f"RESULT main={main_kind} reps={reps} mismatching replays {bad}; side first replay vs "
          f"eager differs at {vs_eager}; per (stream, shape) {sorted(which.items(), key=str)}",
          flush=True)


if __name__ == "__main__":
    main()
