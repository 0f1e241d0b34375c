"""Image-plane projection of scene flow for the 2D metrics (reference: utils/geometry.py:6-65).

`get_batch_2d_flow` projects pc1, pc1 + gt flow and pc1 + predicted flow with the KITTI
left-colour camera (`P_rect_02` of each scene's calib_cam_to_cam/<scene>.txt) when the scene
paths are KITTI's, else with FlyingThings3D's fixed intrinsics (f = -1050, c = (479.5,
269.5)).  Arrays may be NumPy (the reference's arithmetic, float64 calibration broadcast
against float32 points) or torch tensors on any device (the calibration is moved to the
points' device; no host round trip).  The calibration files are KITTI data and are not
shipped: `calib_dir` (or $KDPC_KITTI_CALIB, or `calib_cam_to_cam/` next to this module)."""
import functools
import os
import os.path as osp

import numpy as np
import torch


def calib_dir_default():
    return os.environ.get("KDPC_KITTI_CALIB",
                          osp.join(osp.dirname(osp.abspath(__file__)), "calib_cam_to_cam"))


@functools.lru_cache(maxsize=512)
def read_p_rect_02(path):
    """The 3x4 P_rect_02 matrix (float32) of one calib_cam_to_cam file."""
    with open(path) as fd:
        line = next(ln for ln in fd.readlines() if ln.startswith("P_rect_02"))
    return np.array([float(v) for v in line.split()[1:]], dtype=np.float32).reshape(3, 4)


def kitti_intrinsics(paths, calib_dir=None):
    """Per-scene (f, cx, cy, constx, consty, constz), each (B,1) float64 (f = -P[0,0]).
    The reference builds them as (B,1,1), which against (B,N) coordinates broadcasts to
    (B,B,N) -- every scene's points through every scene's camera.  Its evaluation runs at
    batch_size 1 (config_evaluate_bid_pointconv.yaml), where both agree (up to that extra
    unit axis); (B,1) keeps scene b on camera b for any batch size."""
    cdir = calib_dir or calib_dir_default()
    mats = [read_p_rect_02(osp.join(cdir, osp.split(p)[-1] + ".txt")) for p in paths]
    cols = ([-m[0, 0] for m in mats], [m[0, 2] for m in mats], [m[1, 2] for m in mats],
            [m[0, 3] for m in mats], [m[1, 3] for m in mats], [m[2, 3] for m in mats])
    return tuple(np.array(c)[:, None] for c in cols)


def project_3d_to_2d(pc, f=-1050., cx=479.5, cy=269.5, constx=0, consty=0, constz=0):
    """Pinhole projection of (..., N, 3) points -> (x, y) pixel coordinates."""
    x = (pc[..., 0] * f + cx * pc[..., 2] + constx) / (pc[..., 2] + constz)
    y = (pc[..., 1] * f + cy * pc[..., 2] + consty) / (pc[..., 2] + constz)
    return x, y


def _on(pc, params):
    if not torch.is_tensor(pc):
        return params
    return tuple(torch.as_tensor(p, device=pc.device) for p in params)


def get_batch_2d_flow(pc1, pc2, predicted_pc2, paths, calib_dir=None):
    """pc1, pc2 (= pc1 + gt flow), predicted_pc2 (B,N,3) -> (flow_pred, flow_gt) (B,N,2)."""
    if "KITTI" in paths[0] or "kitti" in paths[0]:
        f, cx, cy, kx, ky, kz = _on(pc1, kitti_intrinsics(paths, calib_dir))
        proj = functools.partial(project_3d_to_2d, f=f, cx=cx, cy=cy, constx=kx, consty=ky,
                                 constz=kz)
    else:
        proj = project_3d_to_2d
    px1, py1 = proj(pc1)
    px2, py2 = proj(predicted_pc2)
    gx2, gy2 = proj(pc2)
    stack = (lambda a, b: torch.stack([a, b], -1)) if torch.is_tensor(pc1) else \
        (lambda a, b: np.concatenate((a[..., None], b[..., None]), axis=-1))
    return stack(px2 - px1, py2 - py1), stack(gx2 - px1, gy2 - py1)
