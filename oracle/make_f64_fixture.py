"""ORACLE — TEST INFRASTRUCTURE ONLY.  Float64 run of the REFERENCE model on the kNN-trace
fixture (tests/golden/model_knntrace_n2048.npz), for the gradient parity tolerance.

The fixture's fp32 reference gradients carry the reference's own fp32 rounding error.  Some
per-parameter gradient sums are near-cancelling (layers just upstream of train-mode
BatchNorm, LeakyReLU pre-activations within rounding of 0), so two correct fp32
implementations can differ there by more than a fixed 1e-4 of |grad|.  This script runs the
same reference code (imported as in make_fixtures.py) in float64, with every knn_point call
replaying the recorded fp32 reference indices in call order and FPS computed by the C
restatement on the (exactly gathered) fp32 coordinates, and stores the float64 gradient
sums: the test then allows the GPU build the reference's own fp32 error |g32 - g64| per
parameter.

    python oracle/make_f64_fixture.py [--n 8192]  -> tests/golden/model_knntrace_n{n}_f64.npz
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
TIE_REL = 1e-4  # |pre-activation| below TIE_REL x the call's scale counts as a near-tie
sys.path.insert(0, HERE)
import make_fixtures as MF  # noqa: E402
from gradproj import projection  # noqa: E402


def main(n=2048, full_grads=None, dtype=torch.float64):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    R = MF.setup_reference()
    g = np.load(os.path.join(MF.GOLDEN, f"model_knntrace_n{n}.npz"))
    calls = [(int(g[f"knn{i}_k"]), g[f"knn{i}_rsum"], g[f"knn{i}_qsum"],
              g[f"knn{i}_idx"].astype(np.int64)) for i in range(int(g["n_calls"]))]
    pos = {"i": 0, "worst": 0.0}

    def replay(nsample, xyz, new_xyz):
        k, rs, qs, idx = calls[pos["i"]]
        pos["i"] += 1
        x = xyz.detach().double().numpy()[0]
        q = new_xyz.detach().double().numpy()[0]
        e = max(np.abs(np.concatenate([x.sum(0), (x ** 2).sum(0)]) - rs).max() / (np.abs(rs).max() + 1),
                np.abs(np.concatenate([q.sum(0), (q ** 2).sum(0)]) - qs).max() / (np.abs(qs).max() + 1))
        assert k == nsample and idx.shape == (q.shape[0], nsample), (pos["i"], k, nsample)
        pos["worst"] = max(pos["worst"], e)
        return torch.from_numpy(idx[None])

    stub = sys.modules["pointnet2_cuda"]
    fps32 = stub.furthest_point_sampling_wrapper

    def fps(b, n_, npoint, points, temp, idx):
        return fps32(b, n_, npoint, points.float(), temp, idx)
    stub.furthest_point_sampling_wrapper = fps
    mods = (R.pcu, sys.modules["pointconv_util2"])
    orig = {m: m.knn_point for m in mods}
    f32 = torch.cuda.FloatTensor
    torch.cuda.FloatTensor = lambda *s: torch.empty(*s, dtype=dtype)
    for m in mods:
        m.knn_point = replay
    # the cost volumes' max over K (CrossLayerLight.cross, pointconv_util.py:1848): record
    # the student's routing -- which neighbour each (point, channel) maximum came from -- in
    # call order, so the GPU test can replay it (a float64 near-tie may route differently
    # from any fp32 evaluation)
    amax = []
    # LeakyReLU near-ties of the same calls: the first activation's pre-activation z0
    # (B, D, K, N1) and the maximum over K of the second activation (B, D, N1), wherever the
    # float64 value lies within TIE_REL of the call's scale of 0 -- the GPU test replays the
    # float64 side there when its own evaluation is not clearly on that side (the derivative
    # jumps from 0.1 to 1 at 0, a discrete choice like the max routing)
    z0ties, z1ties = [], []
    import torch.nn.functional as TF
    pool = TF.max_pool2d

    def ties(v, tau):
        """(flat positions, signs, values) of |v| < tau, v of shape (1, D, *rest)."""
        v = v.detach()[0]
        hit = (v.abs() < tau).nonzero()
        vals = v[tuple(hit.t())] if len(hit) else v.new_zeros(0)
        return hit.numpy().astype(np.int32), np.sign(vals.numpy()).astype(np.int8), vals.numpy()

    def recording_pool(x, kernel_size, *a, **k):
        out, ind = pool(x, kernel_size, *a, return_indices=True, **k)
        n = x.shape[3]
        amax.append((ind[:, :, 0, :] // n).permute(0, 2, 1).to(torch.uint8).numpy())
        scale = float(x.detach().std())
        z1ties.append(ties(out[:, :, 0, :], TIE_REL * scale) + (scale,))  # (d, n)
        return out

    def z0_hook(mod, inputs):
        z0 = inputs[0]
        scale = float(z0.detach().std())
        z0ties.append(ties(z0, TIE_REL * scale) + (scale,))  # positions (d, k, n)
    try:
        pos1, pos2, flow = (torch.from_numpy(g[k]).to(dtype) for k in ("pos1", "pos2", "flow"))
        teacher = MF._synth(R.teacher.PointConvBidirection(), seed=1).to(dtype).eval()
        student = MF._synth(R.student.PointConvBidirection(), seed=2).to(dtype).train()
        with torch.no_grad():
            t_out = teacher(pos1, pos2, pos1, pos2)
        CL = sys.modules["pointconv_util2"].CrossLayerLight
        hooks = [m.relu.register_forward_pre_hook(z0_hook) for m in student.modules()
                 if isinstance(m, CL)]
        TF.max_pool2d = recording_pool
        try:
            s_out = student(pos1, pos2, pos1, pos2)
        finally:
            TF.max_pool2d = pool
            for h in hooks:
                h.remove()
        assert len(z0ties) == len(amax) == len(z1ties), (len(z0ties), len(amax))
        flows, f1i, f2i, _, _, feat1s, feat2s, _ = s_out
        kd = R.loss.biDirection_loss_ht(flows, feat1s, feat2s, f1i, f2i, flow, t_out[0],
                                        t_out[5], t_out[6], t_out[1], t_out[2], 0.3, 0.8, layer=3)
        kd.backward()
    finally:
        for m, fn in orig.items():
            m.knn_point = fn
        torch.cuda.FloatTensor = f32
        stub.furthest_point_sampling_wrapper = fps32
    assert pos["i"] == len(calls), (pos["i"], len(calls))
    named = [(k, p) for k, p in student.named_parameters()]
    proj = [projection(k, p.grad) for k, p in named]
    out = {
        "grad_sum_f64": np.array([float(p.grad.sum()) if p.grad is not None else 0.0
                                  for _, p in named]),
        # two fixed random projections per parameter: sensitive to elementwise errors that
        # cancel in the plain sum (tests compare sum_i g_i r_i against sum_i |g_i r_i|)
        "grad_proj_f64": np.array([p[0] for p in proj]),
        "grad_absproj_f64": np.array([p[1] for p in proj]),
        "kd_f64": kd.detach().numpy(),
        "replay_worst": np.array(pos["worst"]),
    }
    for i in range(4):
        out[f"s_flow{i}_f64"] = flows[i].detach().numpy()
    out["n_amax"] = np.array(len(amax))
    for j, a in enumerate(amax):
        out[f"amax{j}"] = a
    # near-ties, per call: z0 positions as (n, k, d) and z1-max positions as (n, d) in the
    # build's point-major layout, the float64 sign and value, and the call's scale
    out["tie_rel"] = np.array(TIE_REL)
    for j, ((p0, s0, v0, c0), (p1, s1, v1, c1)) in enumerate(zip(z0ties, z1ties)):
        out[f"z0tie{j}_nkd"] = p0[:, ::-1].copy()
        out[f"z0tie{j}_sign"], out[f"z0tie{j}_val"], out[f"z0tie{j}_scale"] = s0, v0, np.array(c0)
        out[f"z1tie{j}_nd"] = p1[:, ::-1].copy()
        out[f"z1tie{j}_sign"], out[f"z1tie{j}_val"], out[f"z1tie{j}_scale"] = s1, v1, np.array(c1)
    print("LeakyReLU near-ties per call (z0, z1 max):",
          [(len(a[0]), len(b[0])) for a, b in zip(z0ties, z1ties)])
    if full_grads:  # every gradient element (diagnostics: tools/grad_gap.py), not committed
        np.savez_compressed(full_grads, **{k: p.grad.numpy() for k, p in student.named_parameters()
                                           if p.grad is not None})
        print("wrote", full_grads)
        return
    path = os.path.join(MF.GOLDEN, f"model_knntrace_n{n}_f64.npz")
    np.savez_compressed(path, **out)
    d = np.abs(out["grad_sum_f64"] - g["grad_sum"]) / (g["grad_abs"] + 1e-12)
    print("replay worst", pos["worst"], "kd32", float(g["kd"]), "kd64", float(out["kd_f64"]))
    print("reference fp32 vs fp64 grad-sum error / |grad|: max", d.max(), "median", np.median(d))
    print("wrote", path)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--full-grads", default=None, help="dump every gradient element here")
    ap.add_argument("--f32", action="store_true", help="run the reference in float32 instead")
    a = ap.parse_args()
    main(a.n, a.full_grads, torch.float32 if a.f32 else torch.float64)
