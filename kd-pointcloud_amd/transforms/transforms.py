"""Per-sample scene-flow transforms (reference: transforms/transforms.py:28-316).

`ProcessData` (evaluation: depth mask + resampling) and `Augmentation` (training: joint
scale / yaw / shift / jitter, a pc2-only yaw / shift, depth mask, resampling) return
(pc1, pc2, sf) exactly as the reference does, drawing from NumPy's global generator in the
reference's order and with its dtypes, so a seeded worker produces the same samples
(tests/test_data_path.py checks this against reference-generated fixtures).  Two reference
quirks are kept on purpose: `jitter_clip: 0.0` in the shipped configs clips the joint jitter
to zero, and the arrays handed in are modified in place by `Augmentation`.

These run on the host inside DataLoader workers (a few hundred microseconds per 8192-point
sample); datasets.DeviceLoader moves the collated batch into HBM on a side stream one step
ahead, so the GPU step never waits on them.  The permutohedral-lattice helpers of the
reference file (`key2int`, `int2key`, `Traverse`: HPLFlowNet leftovers, numba-jitted, not used
by any transform or model here) are not restated.
"""
import numpy as np

from . import functional as F

__all__ = ["Compose", "ToTensor", "ProcessData", "Augmentation"]


class Compose:
    """Reference: transforms.py:29-55."""

    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        body = "".join("\n    {0}".format(t) for t in self.transforms)
        return self.__class__.__name__ + "(" + body + "\n)"


class ToTensor:
    """Reference: transforms.py:58-66."""

    def __call__(self, pic):
        return F.to_tensor(pic) if isinstance(pic, np.ndarray) else pic

    def __repr__(self):
        return self.__class__.__name__ + "()"


def _near(pc1, pc2, depth):
    """Indices of points in front of the depth threshold in both frames."""
    if depth > 0:
        keep = np.logical_and(pc1[:, 2] < depth, pc2[:, 2] < depth)
    else:
        keep = np.ones(pc1.shape[0], dtype=bool)
    return np.where(keep)[0]


def _resample(indices, num_points, no_corr, allow_less_points):
    """The reference's point selection: num_points of the kept indices without replacement
    (pc2 drawn independently when NO_CORR), with replacement when too few remain (or all of
    them when allow_less_points); num_points <= 0 keeps everything."""
    if num_points <= 0:
        return indices, indices
    try:
        i1 = np.random.choice(indices, size=num_points, replace=False, p=None)
        i2 = np.random.choice(indices, size=num_points, replace=False, p=None) if no_corr else i1
    except ValueError:
        if allow_less_points:
            return indices, indices
        i1 = np.random.choice(indices, size=num_points, replace=True, p=None)
        i2 = np.random.choice(indices, size=num_points, replace=True, p=None) if no_corr else i1
    return i1, i2


def _yaw(angle, dtype):
    c, s = np.cos(angle), np.sin(angle)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], dtype=dtype)


def _args_repr(name, groups, depth, no_corr, allow_less, num_points):
    s = name
    for title, args in groups:
        s += "\n({}: \n".format(title) if title == groups[0][0] else "\n{}: \n".format(title)
        for k in sorted(args):
            s += "\t{:10s} {}\n".format(k, args[k])
    s += ("\ndata_process_args: \n\tDEPTH_THRESHOLD: {}\n\tNO_CORR: {}\n\tallow_less_points: {}"
          "\n\tnum_points: {}\n)").format(depth, no_corr, allow_less, num_points)
    return s


class ProcessData:
    """Reference: transforms.py:137-209.  data = [pc1 (N,3+), pc2 (N,3+)] ->
    (pc1 (n,3+), pc2 (n,3+), sf (n,3)) or (None, None, None)."""

    def __init__(self, data_process_args, num_points, allow_less_points):
        self.DEPTH_THRESHOLD = data_process_args["DEPTH_THRESHOLD"]
        self.no_corr = data_process_args["NO_CORR"]
        self.num_points = num_points
        self.allow_less_points = allow_less_points

    def __call__(self, data):
        pc1, pc2 = data
        if pc1 is None:
            return None, None, None
        sf = pc2[:, :3] - pc1[:, :3]
        indices = _near(pc1, pc2, self.DEPTH_THRESHOLD)
        if len(indices) == 0:
            return None, None, None
        i1, i2 = _resample(indices, self.num_points, self.no_corr, self.allow_less_points)
        return pc1[i1], pc2[i2], sf[i1]

    def __repr__(self):
        return ("{}\n(data_process_args: \n\tDEPTH_THRESHOLD: {}\n\tNO_CORR: {}\n"
                "\tallow_less_points: {}\n\tnum_points: {}\n)").format(
                    self.__class__.__name__, self.DEPTH_THRESHOLD, self.no_corr,
                    self.allow_less_points, self.num_points)


class Augmentation:
    """Reference: transforms.py:212-316.  Joint (both frames): scale diag U(lo,hi)^3, yaw
    U(+-degree_range), shift U(+-shift_range)^3, clipped jitter; then pc2 alone: yaw, shift
    (and clipped jitter when the frames correspond); sf = pc2 - pc1 before that jitter;
    depth mask; resampling."""

    def __init__(self, aug_together_args, aug_pc2_args, data_process_args, num_points,
                 allow_less_points=False):
        self.together_args = aug_together_args
        self.pc2_args = aug_pc2_args
        self.DEPTH_THRESHOLD = data_process_args["DEPTH_THRESHOLD"]
        self.no_corr = data_process_args["NO_CORR"]
        self.num_points = num_points
        self.allow_less_points = allow_less_points

    def _jitter(self, args, n):
        return np.clip(args["jitter_sigma"] * np.random.randn(n, 3),
                       -args["jitter_clip"], args["jitter_clip"]).astype(np.float32)

    def __call__(self, data):
        pc1, pc2 = data
        if pc1 is None:
            return None, None, None
        t = self.together_args
        scale = np.diag(np.random.uniform(t["scale_low"], t["scale_high"], 3).astype(np.float32))
        rot = _yaw(np.random.uniform(-t["degree_range"], t["degree_range"]), np.float32)
        joint = scale.dot(rot.T)
        shift = np.random.uniform(-t["shift_range"], t["shift_range"], (1, 3)).astype(np.float32)
        bias = shift + self._jitter(t, pc1.shape[0])
        pc1[:, :3] = pc1[:, :3].dot(joint) + bias
        pc2[:, :3] = pc2[:, :3].dot(joint) + bias

        a = self.pc2_args
        rot2 = _yaw(np.random.uniform(-a["degree_range"], a["degree_range"]), pc1.dtype)
        shift2 = np.random.uniform(-a["shift_range"], a["shift_range"], (1, 3)).astype(np.float32)
        pc2[:, :3] = pc2[:, :3].dot(rot2.T) + shift2
        sf = pc2[:, :3] - pc1[:, :3]
        if not self.no_corr:
            pc2[:, :3] += self._jitter(a, pc1.shape[0])

        indices = _near(pc1, pc2, self.DEPTH_THRESHOLD)
        if len(indices) == 0:
            return None, None, None
        i1, i2 = _resample(indices, self.num_points, self.no_corr, self.allow_less_points)
        return pc1[i1], pc2[i2], sf[i1]

    def __repr__(self):
        return _args_repr(self.__class__.__name__,
                          [("together_args", self.together_args), ("pc2_args", self.pc2_args)],
                          self.DEPTH_THRESHOLD, self.no_corr, self.allow_less_points,
                          self.num_points)
