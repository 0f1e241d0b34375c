"""Scene-flow datasets and the HBM-staging loader.  Reference:
datasets/__init__.py, flyingthings3d_subset{,_min}.py, kitti.py."""
from .flyingthings3d_subset import FlyingThings3DSubset, FlyingThings3DSubsetMin  # noqa: F401
from .kitti import KITTI  # noqa: F401
from .loader import DeviceLoader, collate_scene_flow  # noqa: F401

__all__ = ["FlyingThings3DSubset", "FlyingThings3DSubsetMin", "KITTI", "DeviceLoader",
           "collate_scene_flow"]
