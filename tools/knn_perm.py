"""Is the culled kNN (csrc/knn.hip) independent of the order of its inputs?  The counting
sort leaves the order of refs inside a grid cell to LDS atomics, so it varies with timing;
the result must not.  Here the order is varied on purpose: the kNN calls of one teacher
forward (B=4, N=8192, recorded as tools/knn_race.py does) are rerun with the refs and the
queries of every cloud randomly permuted, the result mapped back to the original indices,
and every row checked against a float64 brute force: K distinct in-range indices whose
largest distance is within rounding of the true K-th distance.  Sequential, one stream.

  python tools/knn_perm.py [perms=20]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kd-pointcloud_amd"))
import torch  # noqa: E402

DEV = "cuda"


def check(idx, x, q, k):
    """rows whose result is not a valid K-nearest set (float64 brute force)"""
    b, n = x.shape[:2]
    bad_range = ((idx < 0) | (idx >= n)).any(-1)
    ii = idx.clamp(0, n - 1).long()
    srt = ii.sort(-1)[0]
    dup = (srt[..., 1:] == srt[..., :-1]).any(-1)
    x64, q64 = x.double(), q.double()
    d_all = torch.cdist(q64, x64) ** 2                       # (B,S,N)
    kth = d_all.topk(k, -1, largest=False)[0][..., -1]       # true K-th distance
    d_got = torch.gather(d_all, 2, ii).max(-1)[0]
    far = d_got > kth + 1e-6 * (1 + kth)
    return bad_range | dup | far, (bad_range.sum().item(), dup.sum().item(), far.sum().item())


def main():
    o = dict(a.split("=") for a in sys.argv[1:])
    perms = int(o.get("perms", 20))
    import kdpc_native as K
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
    g = torch.Generator(device="cpu").manual_seed(7)
    total_bad = 0
    for ci, (x, q, k) in enumerate(rec):
        b, n, s = x.shape[0], x.shape[1], q.shape[1]
        base = K.knn_point(k, x, q)
        torch.cuda.synchronize()
        bad0, why0 = check(base, x, q, k)
        nbad, ndiff, why = 0, 0, [0, 0, 0]
        for r in range(perms):
            pr = torch.stack([torch.randperm(n, generator=g) for _ in range(b)]).to(DEV)
            pq = torch.stack([torch.randperm(s, generator=g) for _ in range(b)]).to(DEV)
            xp = torch.gather(x, 1, pr[..., None].expand(-1, -1, 3)).contiguous()
            qp = torch.gather(q, 1, pq[..., None].expand(-1, -1, 3)).contiguous()
            ip = K.knn_point(k, xp, qp)                      # rows in permuted query order
            # back to original refs and original query rows
            im = torch.gather(pr, 1, ip.clamp(0, n - 1).long().reshape(b, -1)).reshape(b, s, k)
            im = torch.where((ip >= 0) & (ip < n), im, torch.full_like(im, -1))
            out = torch.empty_like(im)
            out.scatter_(1, pq[..., None].expand(-1, -1, k), im)
            bad, w = check(out.int(), x, q, k)
            nbad += int(bad.sum())
            why = [a + c for a, c in zip(why, w)]
            ndiff += int((out.sort(-1)[0] != base.long().sort(-1)[0]).any(-1).sum())
        total_bad += nbad + int(bad0.sum())
        print(f"call {ci} (B={b}, N={n}, S={s}, K={k}): unpermuted invalid rows {int(bad0.sum())} "
              f"{why0}; over {perms} permutations invalid rows {nbad} (range, dup, far) {tuple(why)}; "
              f"rows whose index set differs from the unpermuted one {ndiff}", flush=True)
    print("RESULT invalid rows", total_bad, flush=True)


if __name__ == "__main__":
    main()
