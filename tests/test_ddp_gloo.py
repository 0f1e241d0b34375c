"""CPU, world_size 2 over gloo: the multi-process training path (distill.wrap_ddp +
FlowTrainStep / KDTrainStep) produces exactly the update of the averaged per-shard
gradients (per-replica BatchNorm statistics, as the reference's DataParallel), with the
never-used parameters handled.  The model is the oracle's CPU restatement (the product
model has no CPU path); the DDP code under test is the product's."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N = 2048


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank):
    import synthetic
    return tuple(torch.from_numpy(a) for a in synthetic.ft3d_batch(1, N, seed=50 + rank))


def _models(kd):
    import torch_model as M
    from weights import load_synthetic
    student = load_synthetic(M.PointConvBidirection(), seed=2)
    teacher = load_synthetic(M.PointConvBidirection(), seed=1) if kd else None
    return M, student, teacher


def _sgd(model):
    # plain SGD keeps the update linear in the gradient (Adam's first step is ~lr*sign(g),
    # which would amplify last-bit differences of near-zero gradients)
    return torch.optim.SGD(model.parameters(), lr=0.1)


def _make_step(M, model, teacher, kd):
    import distill
    opt = _sgd(model)
    if kd:
        return distill.KDTrainStep(teacher, model, opt, loss_fn=M.biDirection_loss_ht)
    return distill.FlowTrainStep(model, opt, loss_fn=M.multiScaleLoss)


def _worker(rank, world, port, out_path, kd, paths):
    import sys
    sys.path[:0] = paths
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import distill
    M, student, teacher = _models(kd)
    model = distill.wrap_ddp(student)
    assert isinstance(model, torch.nn.parallel.DistributedDataParallel)
    step = _make_step(M, model, teacher, kd)
    loss = step(*_data(rank))
    assert torch.isfinite(loss).all()
    if rank == 0:
        torch.save({k: v.clone() for k, v in student.state_dict().items()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kd", [False, True], ids=["flow", "kd"])
def test_ddp_step_equals_averaged_shard_gradients(kd):
    import sys
    threads = torch.get_num_threads()
    torch.set_num_threads(2)
    try:
        _check(kd)
    finally:
        torch.set_num_threads(threads)


def _check(kd):
    import sys
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker, args=(2, _port(), out, kd, list(sys.path)), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)

    # single process: gradients of each shard, averaged, then one Adam step
    grads = []
    for rank in range(2):
        M, student, teacher = _models(kd)
        pos1, pos2, flow = _data(rank)
        if kd:
            teacher.eval()
            with torch.no_grad():
                t = teacher(pos1, pos2, pos1, pos2)
            s = student.train()(pos1, pos2, pos1, pos2)
            loss = M.biDirection_loss_ht(s[0], s[5], s[6], s[1], s[2], flow, t[0], t[5], t[6],
                                         t[1], t[2], 0.3, 0.8, layer=3)
        else:
            s = student.train()(pos1, pos2, pos1, pos2)
            loss = M.multiScaleLoss(s[0], flow, s[1])
        loss.backward()
        grads.append({k: (p.grad.clone() if p.grad is not None else None)
                      for k, p in student.named_parameters()})
        if rank == 0:
            bn_state = {k: v.clone() for k, v in student.state_dict().items()}
    M, ref, _ = _models(kd)
    opt = _sgd(ref)
    n_unused = 0
    for k, p in ref.named_parameters():
        g0, g1 = grads[0][k], grads[1][k]
        if g0 is None:
            n_unused += 1
            continue
        p.grad = (g0 + g1) / 2
    opt.step()
    assert n_unused == 80  # bias1/bias2 + WeightNet BN params
    sd = ref.state_dict()
    for k, v in got.items():
        if "running" in k or "num_batches" in k:
            # BN buffers: rank 0's own shard statistics (DataParallel device-0 semantics)
            torch.testing.assert_close(v, bn_state[k], rtol=0, atol=0)
            continue
        torch.testing.assert_close(v, sd[k], rtol=1e-6, atol=1e-6, msg=k)


def test_graphed_step_requires_warmup():
    """GraphedStep lays the flat buffers out in the order the last warm-up backward finalised
    the gradients: warmup=0 is refused up front with a clear message (CPU, no capture)."""
    import distill
    p = torch.nn.Parameter(torch.zeros(3))
    with pytest.raises(ValueError, match="warmup >= 1"):
        distill.GraphedStep(lambda x: p.sum(), [p], torch.optim.SGD([p], lr=0.1),
                            (torch.zeros(1),), warmup=0)
