"""Find an input order for which the culled kNN (csrc/knn.hip) returns a wrong row and dump
everything needed to replay that launch on the CPU (tools/knn_cull_emul.py): the permuted
refs and queries, the workspace the four kernels left (bbox, cell offsets, sorted refs,
chunk boxes, sorted queries, seed windows), the result and the list of wrong rows.

A row is wrong when it holds an out-of-range or repeated index, or misses a ref whose exact
(float64) distance is below the row's largest returned distance by more than the rounding
of the float32 expanded form (2^-19 (|q|^2 + |r|^2) covers it).

  python tools/knn_dump.py [calls=3,5] [perms=40]   -> gpurun_out/race/knn_dump_call<i>.npz
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kd-pointcloud_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

DEV = "cuda"


def wrong_rows(idx, x, q):
    b, n = x.shape[:2]
    k = idx.shape[-1]
    bad = ((idx < 0) | (idx >= n)).any(-1)
    ii = idx.clamp(0, n - 1).long()
    srt = ii.sort(-1)[0]
    bad |= (srt[..., 1:] == srt[..., :-1]).any(-1)
    x64, q64 = x.double(), q.double()
    d_all = torch.cdist(q64, x64) ** 2                                   # (B,S,N)
    d_max = torch.gather(d_all, 2, ii).max(-1)[0]
    tol = 2.0 ** -19 * ((q64 ** 2).sum(-1) + (x64 ** 2).sum(-1).max(-1)[0][:, None])
    member = torch.zeros_like(d_all, dtype=torch.bool).scatter_(2, ii, True)
    missed = (~member & (d_all < (d_max - tol)[..., None])).any(-1)
    return bad | missed


def main():
    o = dict(a.split("=") for a in sys.argv[1:])
    calls = [int(c) for c in o.get("calls", "3,5").split(",")]
    perms = int(o.get("perms", 40))
    import kdpc_native as K
    import synthetic
    from models_bid_pointconv import PointConvBidirection as Teacher
    lib = K.load_library()
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
    g = torch.Generator(device="cpu").manual_seed(11)
    os.makedirs("gpurun_out/race", exist_ok=True)
    for ci in calls:
        x, q, k = rec[ci]
        b, n, s = x.shape[0], x.shape[1], q.shape[1]
        nb = lib.kdpc_knn_workspace_bytes(b, n, s)
        assert nb > 0
        ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
        found = False
        for r in range(perms + 1):
            if r == 0:
                xp, qp = x, q
            else:
                pr = torch.stack([torch.randperm(n, generator=g) for _ in range(b)]).to(DEV)
                pq = torch.stack([torch.randperm(s, generator=g) for _ in range(b)]).to(DEV)
                xp = torch.gather(x, 1, pr[..., None].expand(-1, -1, 3)).contiguous()
                qp = torch.gather(q, 1, pq[..., None].expand(-1, -1, 3)).contiguous()
            idx = torch.empty((b, s, k), dtype=torch.int32, device=DEV)
            dist = torch.empty((b, s, k), dtype=torch.float32, device=DEV)
            rc = lib.kdpc_knn_point_ws(b, n, s, k, xp.data_ptr(), qp.data_ptr(), idx.data_ptr(),
                                       dist.data_ptr(), ws.data_ptr(), nb,
                                       torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            bad = wrong_rows(idx, xp, qp)
            nbad = int(bad.sum())
            print(f"call {ci} (B={b}, N={n}, S={s}, K={k}) order {r}: wrong rows {nbad}",
                  flush=True)
            if nbad and not found:
                found = True
                rows = bad.nonzero().cpu().numpy()
                np.savez(f"gpurun_out/race/knn_dump_call{ci}.npz", xyz=xp.cpu().numpy(),
                         new_xyz=qp.cpu().numpy(), k=k, idx=idx.cpu().numpy(),
                         dist=dist.cpu().numpy(), ws=ws.cpu().numpy(), rows=rows)
                print(f"  dumped; first wrong rows (cloud, query) {rows[:6].tolist()}", flush=True)
            if found and r >= 3:
                break
    print("RESULT done", flush=True)


if __name__ == "__main__":
    main()
