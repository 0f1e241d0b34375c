"""Evaluation on the device and the HBM-staging loader (rank 2) on real
KITTI points from the reference-generated fixture (tests/golden/data_path_ref.npz).

* DeviceLoader on cuda yields exactly the tensors the host DataLoader collates (same seeds).
* evaluate() -- every metric computed and accumulated on the GPU, one host read -- equals the
  reference's NumPy metrics (evaluation_utils / get_batch_2d_flow semantics, checked
  bit-exact against the reference in tests/test_data_path.py) applied per batch to the same
  model outputs, averaged the reference's way."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENES = (1, 2, 3)


@pytest.fixture(scope="module")
def kitti(tmp_path_factory):
    g = np.load(os.path.join(GOLDEN, "data_path_ref.npz"))
    root = tmp_path_factory.mktemp("kitti")
    for s in SCENES:
        d = root / "kitti_processed" / ("%06d" % s)
        d.mkdir(parents=True)
        np.save(d / "pc1.npy", g[f"k{s}_pc1"])
        np.save(d / "pc2.npy", g[f"k{s}_pc2"])
    with open(root / "KITTI_mapping.txt", "w") as fd:
        fd.write("".join(("x\n" if v else "\n") for v in g["mapping_nonempty"]))
    calib = root / "calib"
    calib.mkdir()
    for s in SCENES:
        (calib / ("%06d.txt" % s)).write_text(str(g[f"calib{s}_p_rect_02"]) + "\n")
    return root


def _dataset(root, n):
    import datasets as D
    import transforms as T
    return D.KITTI(train=False, transform=T.ProcessData(dict(DEPTH_THRESHOLD=35., NO_CORR=True),
                                                        n, False),
                   num_points=n, data_root=str(root))


def test_device_loader_stages_same_batches(kitti):
    import datasets as D
    ds = _dataset(kitti, 1024)
    np.random.seed(5)
    host = list(D.DeviceLoader(ds, 1, "cpu"))
    np.random.seed(5)
    dev = list(D.DeviceLoader(ds, 1, "cuda"))
    assert len(host) == len(dev) == 2
    for h, d in zip(host, dev):
        for a, b in zip(h[:5], d[:5]):
            assert b.is_cuda
            assert torch.equal(a, b.cpu())
        assert h[5] == d[5]


def test_evaluate_on_device_matches_reference_metrics(kitti):
    import datasets as D
    import loss_functions
    from evaluate_bid_pointconv import evaluate
    from evaluation_utils import evaluate_2d, evaluate_3d
    from models_bid_lighttoken_res import PointConvBidirection
    from utils import geometry
    torch.manual_seed(0)
    model = PointConvBidirection().cuda().eval()
    ds = _dataset(kitti, 2048)
    np.random.seed(7)
    got = evaluate(model, D.DeviceLoader(ds, 1, "cuda"), calib_dir=str(kitti / "calib"))
    np.random.seed(7)
    rows, seen, tl, te = [], 0, 0.0, 0.0
    with torch.no_grad():
        for pos1, pos2, n1, n2, flow, paths in D.DeviceLoader(ds, 1, "cpu"):
            p1, p2, f = pos1.cuda(), pos2.cuda(), flow.cuda()
            out = model(p1, p2, p1, p2)
            full = out[0][0].permute(0, 2, 1)
            tl += float(loss_functions.multiScaleLoss(out[0], f, out[1]))
            te += float(torch.norm(full - f, dim=2).mean())
            seen += 1
            pc1, sf, pred = pos1.numpy(), flow.numpy(), full.cpu().numpy()
            m3 = evaluate_3d(pred, sf)
            fp, fg = geometry.get_batch_2d_flow(pc1, pc1 + sf, pc1 + pred, paths,
                                                calib_dir=str(kitti / "calib"))
            rows.append([*m3, *evaluate_2d(fp, fg)])
    want = np.mean(np.array(rows, dtype=np.float64), 0)
    keys = ("EPE3D", "ACC3DS", "ACC3DR", "Outliers3D", "EPE2D", "ACC2D")
    np.testing.assert_allclose([got[k] for k in keys], want, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose([got["loss"], got["epe"]], [tl / seen, te / seen], rtol=1e-5)
    assert got["batches"] == 2 and got["samples"] == 2
