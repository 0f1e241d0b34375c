"""Where do the tiled and untiled PointConv backward's dwt differ?  (diagnostic)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402
from test_gpu_fused import _tiled_inputs  # noqa: E402

for (b, n, s, k, d, o) in [(2, 2048, 2048, 9, 125, 128), (1, 1024, 1024, 9, 5, 128)]:
    xyz, center, feats, idx, wt, wl, dy = _tiled_inputs(b, n, s, k, d, o, True, n + k + d)
    ref = K.pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, K.csr_rank_of(idx, n))
    ops = K.load_ops()
    for morton in (False, True):
        order = ops.morton_order(center) if morton else None
        trow, tpair, tsoff, tkey = ops.pc_tile_plan(idx, order, n)
        offsets, perm = ops.csr_build(tkey, n)
        tdst = ops.csr_rank(tkey, offsets, perm, n)
        idx2 = idx.clone()
        tp = K.attach_tile_plan(idx2, n, trow, tpair, tsoff, offsets, tdst.view(tkey.shape))
        got = K.pointconv_bwd_tiled(xyz, center, feats, idx2, wt, wl, dy, tp)
        dw = (got[3] != ref[3]).any(-1).reshape(b * s, k)  # (row, k) pairs that differ
        rows = dw.any(-1).nonzero().flatten()
        print((b, n, s, k, d, o), "morton" if morton else "identity", "pairs differ",
              int(dw.sum()), "of", dw.numel(), "rows", rows[:10].tolist(),
              "max abs", float((got[3] - ref[3]).abs().max()),
              "dcenter eq", bool(torch.equal(got[2], ref[2])),
              "dwl eq", bool(torch.equal(got[4], ref[4])), flush=True)
        if len(rows):
            # tile position of the differing rows
            tr = trow.view(-1).cpu()
            pos = {int(r): i for i, r in enumerate(tr.tolist()) if r >= 0}
            print("   tile slots of differing rows", [pos[int(r)] % 32 for r in rows[:20]],
                  "k of differing pairs", dw[rows[0]].nonzero().flatten().tolist(), flush=True)
