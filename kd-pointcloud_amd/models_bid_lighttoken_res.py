"""Student network — drop-in for the reference's
models_bid_lighttoken_res.PointConvBidirection (models_bid_lighttoken_res.py:14-189).

The reference student has exactly the teacher's graph and channel widths (SURVEY §2a:
7,961,464 parameters and 438 state_dict keys each); it only passes weightnet=16
explicitly.  It is therefore the same class here.
"""
from models_bid_pointconv import PointConvBidirection, multiScaleLoss, scale  # noqa: F401
