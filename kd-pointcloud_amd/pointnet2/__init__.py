"""MI355X drop-in for the reference's `pointnet2` package (pointnet2/pointnet2_utils.py)."""
