"""Print GPU-vs-reference parity numbers for the full model (free-running kNN and with
the reference's neighbour indices replayed).  Run on the GPU box:  python tools/parity_report.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import loss_functions as L  # noqa: E402
import pointconv_util as P  # noqa: E402
from models_bid_pointconv import PointConvBidirection as Net  # noqa: E402
from weights import load_synthetic  # noqa: E402
from test_gpu_model import _KnnReplay  # noqa: E402

DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu().numpy()
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


class _Reversed(_KnnReplay):
    """Same neighbours, K-order reversed: a pure summation-order perturbation."""

    def __call__(self, nsample, xyz, new_xyz):
        return super().__call__(nsample, xyz, new_xyz).flip(-1).contiguous()


def grad_sums(g, knn):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(g[k])).to(DEV)  # noqa: E731
    pos1, pos2, flow = t("pos1"), t("pos2"), t("flow")
    prev = P.set_knn_override(knn)
    try:
        teacher = load_synthetic(Net(), seed=1).to(DEV).eval()
        student = load_synthetic(Net(), seed=2).to(DEV).train()
        with torch.no_grad():
            to = teacher(pos1, pos2, pos1, pos2)
        so = student(pos1, pos2, pos1, pos2)
        kd = L.biDirection_loss_ht(so[0], so[5], so[6], so[1], so[2], flow, to[0], to[5], to[6],
                                   to[1], to[2], 0.3, 0.8, layer=3)
        kd.backward()
    finally:
        P.set_knn_override(prev)
    return {n: float(p.grad.double().sum()) for n, p in student.named_parameters() if p.grad is not None}


def run(g, replay):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(g[k])).to(DEV)  # noqa: E731
    pos1, pos2, flow = t("pos1"), t("pos2"), t("flow")
    prev = P.set_knn_override(_KnnReplay(g) if replay else None)
    try:
        teacher = load_synthetic(Net(), seed=1).to(DEV).eval()
        student = load_synthetic(Net(), seed=2).to(DEV).train()
        with torch.no_grad():
            to = teacher(pos1, pos2, pos1, pos2)
        so = student(pos1, pos2, pos1, pos2)
        msl = L.multiScaleLoss(so[0], flow, so[1])
        kd = L.biDirection_loss_ht(so[0], so[5], so[6], so[1], so[2], flow, to[0], to[5], to[6],
                                   to[1], to[2], 0.3, 0.8, layer=3)
        kd.backward()
    finally:
        P.set_knn_override(prev)
    epe = torch.norm(so[0][0].permute(0, 2, 1) - flow, dim=2).mean()
    out = {f"{tag}_flow{i}": rel(o[0][i], g[f"{tag}_flow{i}"]) for tag, o in (("t", to), ("s", so)) for i in range(4)}
    out["msl"] = rel(msl, g["msl"])
    out["kd"] = rel(kd, g["kd"])
    out["s_epe3d"] = rel(epe, g["s_epe3d"])
    out["s_epe3d_value"] = float(epe)
    # gradient sums vs the reference's, relative to the parameter's |grad| sum; worst 4
    worst = []
    for (name, p), gs, ga in zip(student.named_parameters(), g["grad_sum"], g["grad_abs"]):
        if p.grad is not None and not (name.endswith(".linear.bias") and "pointconv_list" in name):
            worst.append((abs(float(p.grad.double().sum()) - gs) / max(ga, 1e-12), name))
    worst.sort(reverse=True)
    out["grad_worst"] = [f"{r:.1e} {n}" for r, n in worst[:4]]
    return out


if __name__ == "__main__":
    g4 = np.load(os.path.join(ROOT, "tests/golden/model_ref_n4096.npz"))
    g2 = np.load(os.path.join(ROOT, "tests/golden/model_knntrace_n2048.npz"))
    for name, g, rp in (("n4096 free kNN", g4, False), ("n2048 free kNN", g2, False),
                        ("n2048 replayed reference kNN", g2, True)):
        r = run(g, rp)
        print(name, {k: (v if k == "grad_worst" else f"{v:.2e}" if "value" not in k else f"{v:.6f}")
                     for k, v in r.items()})
    for fpc, fcv in ((False, True), (True, False), (False, False)):
        P._FUSED_POINTCONV, P._FUSED_COST_VOLUME = fpc, fcv
        r = run(g2, True)
        print(f"n2048 replayed, fused pointconv={fpc} cost volume={fcv}", r["grad_worst"])
    P._FUSED_POINTCONV = P._FUSED_COST_VOLUME = True
    a, b = grad_sums(g2, _KnnReplay(g2)), grad_sums(g2, _Reversed(g2))
    ga = dict(zip([n for n, _ in Net().named_parameters()], g2["grad_abs"]))
    noise = sorted(((abs(a[n] - b[n]) / max(ga[n], 1e-12), n) for n in a
                    if not (n.endswith(".linear.bias") and "pointconv_list" in n)), reverse=True)
    print("GPU vs GPU, K-order reversed (summation-order noise):", [f"{r:.1e} {n}" for r, n in noise[:6]])
