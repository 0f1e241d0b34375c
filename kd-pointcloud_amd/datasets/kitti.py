"""KITTI scene flow 2015 (HPLFlowNet preprocessing: 200 scenes of pc1.npy / pc2.npy).
Reference: datasets/kitti.py:11-104.

The scene filter is the reference's KITTI_mapping.txt (a scene is kept when its line is
non-empty; 142 of 200).  It is looked up as `mapping_path`, else
`<data_root>/KITTI_mapping.txt`, else the copy shipped next to this module (one line per
scene, "x" where the reference's line is non-empty -- all the filter reads -- generated from
the reference-produced fixture tests/golden/data_path_ref.npz `mapping_nonempty`).  Without
any of them the dataset raises, as the reference does (its open() fails): metrics on all 200
scenes are not comparable with the reference's.  `allow_unfiltered=True` is the explicit
opt-out (every scene kept)."""
import os.path as osp
import warnings

import numpy as np

from ._scenes import SceneFlowDataset, leaf_dirs, load_pair

__all__ = ["KITTI"]


class KITTI(SceneFlowDataset):
    SUBDIR = "kitti_processed"

    def __init__(self, train, transform, num_points, data_root, remove_ground=True,
                 mapping_path=None, allow_unfiltered=False):
        self.root = osp.join(data_root, self.SUBDIR)
        self.train = train
        self.transform = transform
        self.num_points = num_points
        self.remove_ground = remove_ground
        self.allow_unfiltered = allow_unfiltered
        self.mapping_path = mapping_path or next(
            (p for p in (osp.join(data_root, "KITTI_mapping.txt"),
                         osp.join(osp.dirname(osp.abspath(__file__)), "KITTI_mapping.txt"))
             if osp.isfile(p)), None)
        self.samples = self.make_dataset()
        if len(self.samples) == 0:
            raise RuntimeError("Found 0 files in subfolders of: " + self.root + "\n")

    def _repr_lines(self):
        return ["    is removing ground: {}\n".format(self.remove_ground)]

    def make_dataset(self):
        paths = leaf_dirs(osp.realpath(osp.expanduser(self.root)))
        if len(paths) != 200:
            warnings.warn("KITTI: expected 200 scenes, found {}".format(len(paths)))
        if self.mapping_path is None:
            if not self.allow_unfiltered:
                raise FileNotFoundError(
                    "KITTI: KITTI_mapping.txt not found (mapping_path, <data_root>/ or next to "
                    "datasets/kitti.py); it selects the 142 evaluation scenes.  Pass "
                    "allow_unfiltered=True to evaluate every scene instead.")
            warnings.warn("KITTI: no KITTI_mapping.txt; keeping every scene (allow_unfiltered)")
            return paths
        with open(self.mapping_path) as fd:
            lines = [line.strip() for line in fd.readlines()]
        return [p for p in paths if lines[int(osp.split(p)[-1])] != ""]

    def pc_loader(self, path):
        """pc1, pc2 (N,3) float32; ground (y < -1.4 in both frames) removed if asked."""
        pc1, pc2 = load_pair(path)
        if self.remove_ground:
            keep = np.logical_not(np.logical_and(pc1[:, 1] < -1.4, pc2[:, 1] < -1.4))
            pc1, pc2 = pc1[keep], pc2[keep]
        return pc1, pc2
