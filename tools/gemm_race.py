"""Are torch's BLAS GEMMs safe when two streams of one process run them concurrently inside
one HIP graph?  (the KD teacher race: the side stream's Linear output changed after
the fact while a second model ran on the capture stream.)

Each of two streams runs a chain of Linear-shaped GEMMs (the models' forward shapes); the
graph is replayed R times and every output is compared with the first replay's.
  python tools/gemm_race.py [mode=addmm|mm|mm_add|hip] [blas=lt|rocblas] [reps=300] [one=0]
one=1: the same chain on the capture stream only (control).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kd-pointcloud_amd"))
import torch  # noqa: E402

DEV = "cuda"
SHAPES = [(65536, 96, 64), (65536, 64, 64), (16384, 192, 128), (16384, 128, 128),
          (4096, 320, 128), (4096, 128, 128), (2048, 512, 256), (1024, 256, 256),
          (131072, 32, 32), (32768, 64, 32)]


def main():
    o = dict(a.split("=") for a in sys.argv[1:])
    mode, reps = o.get("mode", "addmm"), int(o.get("reps", 300))
    if o.get("blas", "lt") == "rocblas":
        torch.backends.cuda.preferred_blas_library("cublas")
    else:
        torch.backends.cuda.preferred_blas_library("cublaslt")
    print("blas:", torch.backends.cuda.preferred_blas_library(), "mode:", mode, flush=True)
    g = torch.Generator(device="cpu").manual_seed(0)

    def chain_inputs():
        return [(torch.randn(r, i, generator=g).to(DEV), (torch.randn(out, i, generator=g) /
                 i ** 0.5).to(DEV), torch.randn(out, generator=g).to(DEV)) for r, i, out in SHAPES]
    ins = {"side": chain_inputs(), "main": chain_inputs()}

    def lin(x, w, b):
        if mode == "addmm":
            y = torch.empty(x.shape[0], w.shape[0], device=DEV)
            torch.addmm(b, x, w.t(), out=y)
            return y
        if mode == "mm":
            return torch.mm(x, w.t())
        if mode == "mm_add":
            return torch.mm(x, w.t()) + b
        raise ValueError(mode)

    def chain(k):
        return [lin(x, w, b) for x, w, b in ins[k]]

    side = torch.cuda.Stream()

    def body():
        cur = torch.cuda.current_stream()
        res = {}
        if o.get("one", "0") != "1":
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                res["side"] = chain("side")
        res["main"] = chain("main")
        if "side" in res:
            cur.wait_stream(side)
        return res

    body()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        outs = body()
    gr.replay()
    torch.cuda.synchronize()
    ref = {k: [t.clone() for t in v] for k, v in outs.items()}
    eager = {k: chain(k) for k in outs}
    torch.cuda.synchronize()
    vs_eager = {k: sum(not torch.equal(a, c) for a, c in zip(ref[k], eager[k])) for k in outs}
    bad = {k: 0 for k in outs}
    which = {}
    for r in range(reps):
        gr.replay()
        torch.cuda.synchronize()
        for k in outs:
            d = [i for i, (a, c) in enumerate(zip(outs[k], ref[k])) if not torch.equal(a, c)]
            if d:
                bad[k] += 1
                for i in d:
                    which[(k, i)] = which.get((k, i), 0) + 1
    print(f"RESULT mode={mode} blas={o.get('blas', 'lt')} one={o.get('one', '0')} reps={reps} "
          f"mismatching replays {bad}; first replay vs eager (outputs differing) {vs_eager}; "
          f"per (stream, GEMM) {sorted(which.items())}", flush=True)


if __name__ == "__main__":
    main()
