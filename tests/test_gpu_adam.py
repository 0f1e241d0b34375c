"""kdpc_adam_step (csrc/adam.hip) against torch's fused Adam, the optimizer the graphed step
replaced with it: bit-identical parameters and moments over several steps, with the
training configuration (L2 weight decay 1e-4, betas (0.9, 0.999), eps 1e-8, a device lr
tensor, capturable step counters; distill.make_optimizer, distilTrain.py:134-135)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _adam_pair(n, seed, wd=1e-4, maximize=False, lr=1e-3):
    g = torch.Generator(device="cpu").manual_seed(seed)
    p0 = (torch.randn(n, generator=g) * 0.1).to(DEV)
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([ref], lr=torch.tensor(lr, device=DEV), betas=(0.9, 0.999), eps=1e-8,
                           weight_decay=wd, maximize=maximize, fused=True, capturable=True)
    P, M, V = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    step = torch.zeros((), device=DEV)
    lr_t = torch.tensor(lr, device=DEV)
    return g, ref, opt, P, M, V, step, lr_t


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_adam_step_matches_torch_fused_adam(mode):
    """Mismatching elements per step for the four compiled forms (mode bit 0: the double
    expressions contracted as clang does by default; bit 1: fast f32 division / sqrt); the
    form kdpc_native.ADAM_MODE selects must match torch bit for bit.  Measured (round 6):
    mode 1 0 mismatches in 6 steps x 12.6 M values; mode 0 7-20 K per step from step 2;
    modes 2 / 3 82 K from step 1."""
    import kdpc_native as K
    n = 1 << 22
    g, ref, opt, P, M, V, step, lr_t = _adam_pair(n, 3)
    bad = []
    for it in range(6):
        # gradients over many magnitudes, some exactly zero
        G = (torch.randn(n, generator=g) * torch.exp(torch.randn(n, generator=g) * 4)).to(DEV)
        G[::97] = 0.0
        ref.grad = G.clone()
        opt.step()
        step.add_(1)
        K.adam_step(P, G, M, V, lr_t, step, 0.9, 0.999, 1e-8, 1e-4, False, mode=mode)
        st = opt.state[ref]
        bad.append(int((P != ref.detach()).sum() + (M != st["exp_avg"]).sum()
                       + (V != st["exp_avg_sq"]).sum()))
    print(f"mode={mode}: mismatching elements per step {bad}")
    if mode == K.ADAM_MODE:
        assert sum(bad) == 0, bad


def test_adam_step_options_and_graph_replay():
    """maximize, no weight decay, an lr changed between replays of a captured step: the
    kernel reads lr / step from the device each replay."""
    import kdpc_native as K
    n = 4096 * 3
    g, ref, opt, P, M, V, step, lr_t = _adam_pair(n, 5, wd=0.0, maximize=True)
    G = torch.empty(n, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        K.adam_step(P.clone(), G.normal_(), M.clone(), V.clone(), lr_t, step + 1, 0.9, 0.999,
                    1e-8, 0.0, True)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step.add_(1)
        K.adam_step(P, G, M, V, lr_t, step, 0.9, 0.999, 1e-8, 0.0, True)
    for it in range(4):
        lr = 1e-3 * (it + 1)
        lr_t.fill_(lr)
        opt.param_groups[0]["lr"].fill_(lr)
        G.copy_(torch.randn(n, generator=g).to(DEV))
        ref.grad = G.clone()
        opt.step()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(P, ref.detach()), it
        assert torch.equal(M, opt.state[ref]["exp_avg"]), it
