"""Localise fused-vs-unfused differences of the model's wide cost-volume backward (N=2048
trace fixture): per call, the queries whose dp1 rows differ and what is special about them
(diagnostic).

    python tools/cv_localise.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kd-pointcloud_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def f64_grads(x1, x2, idx, p1, p2, wpos, bpos, w1, b1, am, gout):
    """Float64 torch formulation with the given routing."""
    d = lambda t: t.detach().double().clone().requires_grad_(True)  # noqa: E731
    X1, X2, P1, P2, WP, BP, W1, B1 = (d(t) for t in (x1, x2, p1, p2, wpos, bpos, w1, b1))
    B, N1, K = idx.shape
    bi = torch.arange(B, device=idx.device).view(B, 1, 1)
    il = idx.long()
    dirn = X2[bi, il] - X1.unsqueeze(2)
    h0 = torch.nn.functional.leaky_relu(P2[bi, il] + P1.unsqueeze(2) + dirn @ WP.t() + BP, 0.1)
    z = torch.nn.functional.leaky_relu(h0 @ W1.t() + B1, 0.1)  # (B,N1,K,D)
    out = torch.gather(z, 2, am.long().unsqueeze(2)).squeeze(2)
    out.backward(gout.double())
    return [P1.grad, X1.grad, W1.grad, B1.grad, WP.grad, BP.grad, P2.grad, X2.grad]


def main():
    import pointconv_util as P
    import test_gpu_model as T
    import kdpc_native as K
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_knntrace_n2048.npz"))
    calls = []
    orig = P._CostVolume.apply

    def rec(*a):
        if a[3].shape[-1] >= 128:
            calls.append([t.detach().clone() if torch.is_tensor(t) else t for t in a])
        return orig(*a)
    P._CostVolume.apply = rec
    try:
        T._run_models(g, T._KnnReplay(g))
    finally:
        P._CostVolume.apply = orig
    for ci, a in enumerate(calls):
        x1, x2, idx, p1, p2, wpos, bpos, w1, b1 = a[:9]
        out, am = K.cost_volume_fwd(x1, x2, idx, p1, p2, wpos, bpos, w1, b1)
        torch.manual_seed(5)
        gout = torch.randn_like(out)
        dp1, dp2, dx1, dx2, dpar = K.cost_volume_bwd_csr(x1, x2, idx, p1, p2, wpos, bpos, w1,
                                                         out, am, gout)
        D = w1.shape[0]
        ref = f64_grads(x1, x2, idx, p1, p2, wpos, bpos, w1, b1, am, gout)
        rdp1, rdx1, rdw1, rdb1 = ref[0], ref[1], ref[2], ref[3]
        err = (dp1.double() - rdp1).abs().amax(-1).view(-1)
        scale = float(rdp1.abs().max())
        bad = torch.nonzero(err > 1e-5 * scale).view(-1)
        db1 = dpar[D * D:D * D + D].double()
        print(f"call {ci} p1 {tuple(p1.shape)}: dp1 bad queries {bad.numel()} of {err.numel()} "
              f"(max {float(err.max()):.3e}, scale {scale:.3e}); db1 max|diff| "
              f"{float((db1 - rdb1).abs().max()):.3e} scale {float(rdb1.abs().max()):.3e}; "
              f"dw1 max|diff| {float((dpar[:D * D].view(D, D).double() - rdw1).abs().max()):.3e}",
              flush=True)
        if bad.numel():
            B, N1, Kk = idx.shape
            qs = bad[:12].tolist()
            print("   bad q:", qs, "wg (qpw=2):", sorted({q // 2 for q in bad.tolist()})[:20])
            for q in qs[:4]:
                b, n = divmod(q, N1)
                row = idx[b, n].tolist()
                print(f"   q {q}: dup nbrs {len(row) - len(set(row))}, am hist "
                      f"{np.bincount(am[b, n].cpu().numpy(), minlength=Kk).tolist()}, "
                      f"out>0 {int((out[b, n] > 0).sum())}, "
                      f"|gout| {float(gout[b, n].abs().max()):.3e}, "
                      f"worst ch {int((dp1[b, n].double() - rdp1[b, n]).abs().argmax())}")


if __name__ == "__main__":
    main()
