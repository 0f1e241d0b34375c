"""CPU: host-side logic of the drop-in modules (construction, state_dict compatibility
with the reference, API surface) and the no-CPU-fallback rule."""
import numpy as np
import pytest
import torch

import kdpc_native


def test_state_dict_keys_match_reference(golden):
    from models_bid_lighttoken_res import PointConvBidirection as Student
    from models_bid_pointconv import PointConvBidirection as Teacher
    keys = list(golden("model_ref_n4096.npz")["state_keys"])
    for cls in (Teacher, Student):
        m = cls()
        assert list(m.state_dict().keys()) == keys
        assert sum(p.numel() for p in m.parameters()) == int(golden("model_ref_n4096.npz")["n_params"])


def test_reference_weights_load_into_product_and_oracle():
    import torch_model as M
    from models_bid_pointconv import PointConvBidirection
    from weights import synthetic_state_dict
    ref_sd = synthetic_state_dict(M.PointConvBidirection().state_dict(), seed=4)
    m = PointConvBidirection()
    m.load_state_dict(ref_sd)  # strict
    for k, v in m.state_dict().items():
        assert torch.equal(v, ref_sd[k]), k


def test_no_cpu_fallback():
    from models_bid_pointconv import PointConvBidirection
    x = torch.zeros(1, 2048, 3)
    with pytest.raises(kdpc_native.KdpcError):
        PointConvBidirection()(x, x, x, x)
    import pointconv_util as P
    with pytest.raises(kdpc_native.KdpcError):
        P.knn_point(4, torch.zeros(1, 16, 3), torch.zeros(1, 8, 3))


def test_public_api_surface():
    import loss_functions as L
    import pointconv_util as P
    import pointconv_util2 as P2
    import pointnet2_cuda
    from pointnet2 import pointnet2_utils as U
    for name in ("Conv1d", "Conv2d", "square_distance", "knn_point", "index_points_gather",
                 "index_points_group", "group", "group_query", "WeightNet", "PointConv",
                 "PointConvD", "CrossLayerLight", "FlowEmbeddingLayer", "PointConvFlow",
                 "PointWarping", "UpsampleFlow", "SceneFlowEstimatorResidual"):
        assert hasattr(P, name) and getattr(P2, name) is getattr(P, name), name
    for name in ("furthest_point_sample", "gather_operation", "three_nn", "three_interpolate",
                 "grouping_operation", "ball_query", "QueryAndGroup", "GroupAll"):
        assert hasattr(U, name), name
    for name in ("ball_query_wrapper", "group_points_wrapper", "group_points_grad_wrapper",
                 "gather_points_wrapper", "gather_points_grad_wrapper",
                 "furthest_point_sampling_wrapper", "three_nn_wrapper",
                 "three_interpolate_wrapper", "three_interpolate_grad_wrapper"):
        assert callable(getattr(pointnet2_cuda, name)), name
    for name in ("multiScaleLoss", "biDirection_loss_ht", "cross_biDirection_loss_ht",
                 "loss_fn_kd_2", "biDirectionLoss", "loss_fn_ht", "cross_loss",
                 "attentiveImitationLoss"):
        assert callable(getattr(L, name)), name


def test_weightnet_channel_last_equals_conv_layout():
    import pointconv_util as P
    torch.manual_seed(0)
    w = P.WeightNet(3, 16)
    x = torch.randn(2, 3, 9, 50)
    a = w(x)                                        # (B,16,K,N) reference layout
    b = w.channel_last(x.permute(0, 3, 2, 1))       # (B,N,K,16)
    torch.testing.assert_close(b.permute(0, 3, 2, 1), a, rtol=1e-5, atol=1e-6)


def test_synthetic_pairs_deterministic_and_shaped():
    import synthetic
    a = synthetic.ft3d_batch(2, 1024, seed=3)
    b = synthetic.ft3d_batch(2, 1024, seed=3)
    for x, y in zip(a, b):
        assert x.shape == (2, 1024, 3) and x.dtype == np.float32
        np.testing.assert_array_equal(x, y)
    assert 2.0 < a[0][..., 2].min() and a[0][..., 2].max() < 40.0
