"""Synthetic FlyingThings3D-shaped scene-flow pairs.

No dataset is reachable offline, so inputs are generated: a scene of planar rectangles
(centres x~U(-12,12), y~U(-8,8), z~U(5,35) -- the DEPTH_THRESHOLD=35 range of
transforms.py:151-153 -- random normals, sides U(1,8)), each moved rigidly (translation
N(0, 0.5^2) per axis + a small yaw about its centre).  pc1 = N points sampled without
replacement from a dense 4N-point surface sample, gt = their flow; pc2 = an INDEPENDENT
sample of the moved surface (NO_CORR=True, transforms.py:163-166); jitter sigma=0.01
(config_train_kd_pointconv.yaml:46).  color = xyz (datasets/flyingthings3d_subset.py:50-52).
Deterministic per (seed, pair).
"""
import numpy as np

N_PATCHES = 12


def _frame(rng):
    n = rng.normal(size=3)
    n /= np.linalg.norm(n)
    a = np.cross(n, [0.0, 1.0, 0.0] if abs(n[1]) < 0.9 else [1.0, 0.0, 0.0])
    a /= np.linalg.norm(a)
    b = np.cross(n, a)
    return a, b


def ft3d_pair(n_points, seed=0, pair=0):
    """-> pos1 (N,3), pos2 (N,3), flow (N,3) float32."""
    rng = np.random.default_rng([seed, pair])
    centres = np.stack([rng.uniform(-12, 12, N_PATCHES), rng.uniform(-8, 8, N_PATCHES),
                        rng.uniform(5, 35, N_PATCHES)], 1)
    sides = rng.uniform(1, 8, (N_PATCHES, 2))
    area = sides[:, 0] * sides[:, 1]
    dense = 4 * n_points
    counts = rng.multinomial(dense, area / area.sum())
    pts, moved = [], []
    for p in range(N_PATCHES):
        a, b = _frame(rng)
        u = rng.uniform(-0.5, 0.5, (counts[p], 2)) * sides[p]
        surf = centres[p] + u[:, :1] * a + u[:, 1:] * b
        t = rng.normal(0.0, 0.5, 3)
        yaw = rng.normal(0.0, 0.05)
        c, s = np.cos(yaw), np.sin(yaw)
        rot = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
        mv = (surf - centres[p]) @ rot.T + centres[p] + t
        pts.append(surf)
        moved.append(mv)
    pts = np.concatenate(pts, 0)
    moved = np.concatenate(moved, 0)
    i1 = rng.choice(dense, n_points, replace=False)
    i2 = rng.choice(dense, n_points, replace=False)
    pos1 = pts[i1] + rng.normal(0.0, 0.01, (n_points, 3))
    flow = moved[i1] - pts[i1]
    pos2 = moved[i2] + rng.normal(0.0, 0.01, (n_points, 3))
    return pos1.astype(np.float32), pos2.astype(np.float32), flow.astype(np.float32)


def ft3d_batch(batch, n_points, seed=0, first_pair=0):
    """-> pos1, pos2, flow each (B,N,3) float32 (numpy)."""
    out = [ft3d_pair(n_points, seed, first_pair + i) for i in range(batch)]
    return tuple(np.stack([o[k] for o in out], 0) for k in range(3))
