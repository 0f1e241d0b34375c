"""Data path and evaluation metrics vs fixtures produced by the
REFERENCE's own code (oracle/make_fixtures.py `data`) on a strided subsample of real KITTI
scenes: loaders (ground removal, mapping filter, FT3D sign flips), seeded ProcessData /
Augmentation (bit-exact: same NumPy draws in the same order), a seeded dataset item, and the
3D / 2D metrics with KITTI calibration and FT3D intrinsics.  CPU only."""
import os

import numpy as np
import pytest
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENES = (1, 2, 3)


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "data_path_ref.npz"))


@pytest.fixture(scope="module")
def kitti_root(g, tmp_path_factory):
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
        (calib / ("%06d.txt" % s)).write_text("calib_time: x\n" + str(g[f"calib{s}_p_rect_02"]) + "\n")
    return root


def test_loaders(g, kitti_root):
    import datasets as D
    for s in SCENES:
        d = str(kitti_root / "kitti_processed" / ("%06d" % s))
        a, b = D.KITTI.pc_loader(type("K", (), {"remove_ground": True})(), d)
        np.testing.assert_array_equal(a, g[f"k{s}_noground_pc1"])
        np.testing.assert_array_equal(b, g[f"k{s}_noground_pc2"])
        a, b = D.FlyingThings3DSubset.pc_loader(None, d)
        np.testing.assert_array_equal(a, g[f"k{s}_ft3d_pc1"])
        np.testing.assert_array_equal(b, g[f"k{s}_ft3d_pc2"])


def test_kitti_dataset_item(g, kitti_root):
    import datasets as D
    import transforms as T
    ds = D.KITTI(train=False, transform=T.ProcessData(dict(DEPTH_THRESHOLD=35., NO_CORR=True),
                                                      2048, False),
                 num_points=2048, data_root=str(kitti_root))
    assert len(ds) == int(g["ds_len"])  # scene 1 is filtered out by the mapping
    np.random.seed(300)
    item = ds[len(ds) - 1]
    for j, k in enumerate(("pos1", "pos2", "norm1", "norm2", "flow")):
        np.testing.assert_array_equal(item[j], g[f"ds_{k}"], err_msg=k)
    assert os.path.basename(item[5]) == str(g["ds_scene"])
    assert "KITTI" in repr(ds)


def test_ft3d_scene_count_checked(tmp_path):
    import datasets as D
    (tmp_path / "FlyingThings3D_subset_processed_35m" / "val" / "0000000").mkdir(parents=True)
    with pytest.raises(RuntimeError):
        D.FlyingThings3DSubset(False, None, 8192, str(tmp_path))


@pytest.mark.parametrize("case", ["pd_nocorr", "pd_corr", "pd_replace", "pd_allowless",
                                  "pd_nodepth", "pd_all"])
def test_process_data_seeded(g, case):
    import transforms as T
    base1, base2 = g["k2_noground_pc1"], g["k2_noground_pc2"]
    n_avail = int(np.logical_and(base1[:, 2] < 35, base2[:, 2] < 35).sum())
    spec = {"pd_nocorr": (dict(DEPTH_THRESHOLD=35., NO_CORR=True), 2048, False),
            "pd_corr": (dict(DEPTH_THRESHOLD=35., NO_CORR=False), 2048, False),
            "pd_replace": (dict(DEPTH_THRESHOLD=35., NO_CORR=True), n_avail + 100, False),
            "pd_allowless": (dict(DEPTH_THRESHOLD=35., NO_CORR=True), n_avail + 100, True),
            "pd_nodepth": (dict(DEPTH_THRESHOLD=0., NO_CORR=True), 1024, False),
            "pd_all": (dict(DEPTH_THRESHOLD=35., NO_CORR=True), 0, False)}
    i = list(spec).index(case)
    dp, npts, allow = spec[case]
    np.random.seed(100 + i)
    r = T.ProcessData(dp, npts, allow)([base1.copy(), base2.copy()])
    for j, k in enumerate(("pc1", "pc2", "sf")):
        np.testing.assert_array_equal(r[j], g[f"{case}_{k}"], err_msg=k)


@pytest.mark.parametrize("case", ["aug_cfg_nocorr", "aug_clip_corr"])
def test_augmentation_seeded(g, case):
    import transforms as T
    together = dict(degree_range=0.1745329252, shift_range=1., scale_low=0.95, scale_high=1.05,
                    jitter_sigma=0.01, jitter_clip=0.00)
    spec = {"aug_cfg_nocorr": (together, dict(degree_range=0., shift_range=0.3,
                                              jitter_sigma=0.01, jitter_clip=0.00), True),
            "aug_clip_corr": (dict(together, jitter_clip=0.02),
                              dict(degree_range=0.1, shift_range=0.3, jitter_sigma=0.01,
                                   jitter_clip=0.05), False)}
    ta, pa, nc = spec[case]
    np.random.seed(200 + list(spec).index(case))
    r = T.Augmentation(ta, pa, dict(DEPTH_THRESHOLD=35., NO_CORR=nc), 2048)(
        [g["k2_noground_pc1"].copy(), g["k2_noground_pc2"].copy()])
    for j, k in enumerate(("pc1", "pc2", "sf")):
        np.testing.assert_array_equal(r[j], g[f"{case}_{k}"], err_msg=k)


def test_transform_rejects_empty():
    import transforms as T
    far = np.full((10, 3), 50.0, np.float32)
    assert T.ProcessData(dict(DEPTH_THRESHOLD=35., NO_CORR=True), 4, False)([far, far]) == \
        (None, None, None)
    assert T.ProcessData(dict(DEPTH_THRESHOLD=35., NO_CORR=True), 4, False)([None, None]) == \
        (None, None, None)


def test_metrics_3d(g):
    from evaluation_utils import evaluate_3d
    got = np.array(evaluate_3d(g["m_pred"], g["m_gt"]), dtype=np.float64)
    np.testing.assert_array_equal(got, g["m_3d"])
    t = [float(v) for v in evaluate_3d(torch.from_numpy(g["m_pred"]), torch.from_numpy(g["m_gt"]))]
    np.testing.assert_allclose(t, g["m_3d"], rtol=1e-6)


def test_metrics_2d(g, kitti_root):
    from evaluation_utils import evaluate_2d
    from utils import geometry
    pc1, gt, pred = g["m_pc1"], g["m_gt"], g["m_pred"]
    calib = str(kitti_root / "calib")
    for j, s in enumerate(SCENES[-2:]):
        sl = slice(j, j + 1)
        path = ["/x/kitti_processed/%06d" % s]
        fp, fg = geometry.get_batch_2d_flow(pc1[sl], pc1[sl] + gt[sl], pc1[sl] + pred[sl], path,
                                            calib_dir=calib)
        want_p = g[f"m_kitti{j}_flow_pred"].reshape(fp.shape)
        want_g = g[f"m_kitti{j}_flow_gt"].reshape(fg.shape)
        np.testing.assert_array_equal(fp, want_p)
        np.testing.assert_array_equal(fg, want_g)
        np.testing.assert_allclose(np.array(evaluate_2d(fp, fg)), g[f"m_kitti{j}_2d"], rtol=1e-12)
        tp, tg = geometry.get_batch_2d_flow(*(torch.from_numpy(a[sl]) for a in
                                              (pc1, pc1 + gt, pc1 + pred)), path, calib_dir=calib)
        np.testing.assert_allclose(tp.numpy(), want_p, rtol=1e-9)
        np.testing.assert_allclose([float(v) for v in evaluate_2d(tp, tg)], g[f"m_kitti{j}_2d"],
                                   rtol=1e-6)
    # a batch of two KITTI scenes: each through its own camera
    paths = ["/x/kitti_processed/%06d" % s for s in SCENES[-2:]]
    fp, _ = geometry.get_batch_2d_flow(pc1, pc1 + gt, pc1 + pred, paths, calib_dir=calib)
    for j in range(2):
        np.testing.assert_array_equal(fp[j], g[f"m_kitti{j}_flow_pred"].reshape(fp[j].shape))
    paths = ["/d/FlyingThings3D_subset_processed_35m/val/0", "/d/FlyingThings3D_subset/val/1"]
    fp, fg = geometry.get_batch_2d_flow(pc1, pc1 + gt, pc1 + pred, paths)
    np.testing.assert_array_equal(fp, g["m_ft3d_flow_pred"])
    np.testing.assert_array_equal(fg, g["m_ft3d_flow_gt"])
    np.testing.assert_allclose(np.array(evaluate_2d(fp, fg)), g["m_ft3d_2d"], rtol=1e-12)


def test_device_loader_cpu(g, kitti_root):
    import datasets as D
    import transforms as T
    ds = D.KITTI(train=False, transform=T.ProcessData(dict(DEPTH_THRESHOLD=35., NO_CORR=True),
                                                      1024, False),
                 num_points=1024, data_root=str(kitti_root))
    batches = list(D.DeviceLoader(ds, 2, "cpu"))
    assert len(batches) == 1
    pos1, pos2, n1, n2, flow, paths = batches[0]
    assert pos1.shape == (2, 1024, 3) and pos1.dtype == torch.float32
    assert torch.equal(pos1, n1) and torch.equal(pos2, n2)
    assert [os.path.basename(p) for p in paths] == ["000002", "000003"]
