"""FlyingThings3D subset (HPLFlowNet preprocessing).  Reference:
datasets/flyingthings3d_subset.py:11-103 and flyingthings3d_subset_min.py (the same loader
over a smaller tree).

Differences, deliberate: an unexpected scene count raises RuntimeError instead of printing
and calling sys.exit(1); pptk (imported but unused by the reference) is not needed."""
import os.path as osp

from ._scenes import SceneFlowDataset, leaf_dirs, load_pair

__all__ = ["FlyingThings3DSubset", "FlyingThings3DSubsetMin"]


class FlyingThings3DSubset(SceneFlowDataset):
    SUBDIR = "FlyingThings3D_subset_processed_35m"
    EXPECTED = {True: 19640, False: 3824}  # train / val scene counts of the full subset

    def __init__(self, train, transform, num_points, data_root, full=True):
        self.root = osp.join(data_root, self.SUBDIR)
        self.train = train
        self.transform = transform
        self.num_points = num_points
        self.samples = self.make_dataset(full)
        if len(self.samples) == 0:
            raise RuntimeError("Found 0 files in subfolders of: " + self.root + "\n")

    def _repr_lines(self):
        return ["    is training: {}\n".format(self.train)]

    def make_dataset(self, full):
        root = osp.join(osp.realpath(osp.expanduser(self.root)), "train" if self.train else "val")
        paths = leaf_dirs(root)
        want = self.EXPECTED[bool(self.train)]
        if want is not None and len(paths) != want:
            raise RuntimeError("{}: found {} scenes under {}, expected {}".format(
                self.__class__.__name__, len(paths), root, want))
        return paths if full else paths[::4]

    def pc_loader(self, path):
        """pc1, pc2 (N,3) float32 with x and z negated (the subset's camera convention)."""
        pc1, pc2 = load_pair(path)
        for pc in (pc1, pc2):
            pc[..., -1] *= -1
            pc[..., 0] *= -1
        return pc1, pc2


class FlyingThings3DSubsetMin(FlyingThings3DSubset):
    SUBDIR = "FlyingThings3D_subset_processed_min"
    EXPECTED = {True: 4504, False: 451}
