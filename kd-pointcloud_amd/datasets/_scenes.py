"""Shared pieces of the scene-flow datasets: leaf-directory discovery, the 6-tuple item and
the None-retry rule of the reference loaders (flyingthings3d_subset.py:36-50,
kitti.py:36-46)."""
import os

import numpy as np
import torch.utils.data as data


def leaf_dirs(root):
    """Sorted directories with no subdirectories below `root` (one scene each)."""
    return [d for d, sub, _ in sorted(os.walk(root)) if len(sub) == 0]


def load_pair(path):
    """pc1.npy / pc2.npy of one scene (float32 (N,3)); plain arrays only, no pickles."""
    pc1 = np.load(os.path.join(path, "pc1.npy"), allow_pickle=False)
    pc2 = np.load(os.path.join(path, "pc2.npy"), allow_pickle=False)
    return pc1, pc2


class SceneFlowDataset(data.Dataset):
    """Item = (pc1, pc2, norm1, norm2, sf, path) with norm = the points themselves (the
    reference feeds xyz as the 'colour' input; its normal estimation is commented out).  A
    sample the transform rejects (None) is replaced by a uniformly drawn other index, as in
    the reference."""

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        while True:
            pc1, pc2 = self.pc_loader(self.samples[index])
            p1, p2, sf = self.transform([pc1, pc2])
            if p1 is not None:
                return p1, p2, p1, p2, sf, self.samples[index]
            index = np.random.choice(range(len(self)))

    def _repr_lines(self):
        return []

    def __repr__(self):
        s = "Dataset " + self.__class__.__name__ + "\n"
        s += "    Number of datapoints: {}\n".format(len(self))
        s += "    Number of points per point cloud: {}\n".format(self.num_points)
        s += "".join(self._repr_lines())
        s += "    Root Location: {}\n".format(self.root)
        tmp = "    Transforms (if any): "
        s += "{0}{1}\n".format(tmp, self.transform.__repr__().replace("\n", "\n" + " " * len(tmp)))
        return s
