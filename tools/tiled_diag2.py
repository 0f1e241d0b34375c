"""Is the untiled PointConv backward's dwt invariant under a permutation of the rows?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import kdpc_native as K  # noqa: E402
from test_gpu_fused import _tiled_inputs  # noqa: E402

b, n, s, k, d, o = 1, 1024, 1024, 9, 5, 128
xyz, center, feats, idx, wt, wl, dy = _tiled_inputs(b, n, s, k, d, o, True, n + k + d)
ref = K.pointconv_bwd(xyz, center, feats, idx, wt, wl, dy, K.csr_rank_of(idx, n))
pi = torch.randperm(s, generator=torch.Generator().manual_seed(1)).to("cuda")
c2, i2, w2, d2 = (t[:, pi].contiguous() for t in (center, idx, wt, dy))
got = K.pointconv_bwd(xyz, c2, feats, i2, w2, wl, d2, K.csr_rank_of(i2, n))
print("dwt perm-invariant:", bool(torch.equal(got[3], ref[3][:, pi])),
      "dcenter:", bool(torch.equal(got[2], ref[2][:, pi])),
      "max abs dwt", float((got[3] - ref[3][:, pi]).abs().max()), flush=True)
y1 = K.pointconv_fwd(xyz, center, feats, idx, wt, wl, torch.zeros(o, device="cuda"))
y2 = K.pointconv_fwd(xyz, c2, feats, i2, w2, wl, torch.zeros(o, device="cuda"))
print("fwd perm-invariant:", bool(torch.equal(y2, y1[:, pi])), flush=True)
