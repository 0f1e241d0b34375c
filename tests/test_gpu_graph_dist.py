"""The multi-rank GraphedStep on ONE GPU.

* world size 2 over gloo (two processes share cuda:0; gloo accepts device tensors): the
  "serial" schedule (graph A fwd+bwd -> eager flat all-reduce -> graph B mean + flat Adam).
  Each rank trains on its own batch; after the steps both ranks hold identical parameters,
  equal to a single-process eager step on the averaged gradient of the two batches -- for
  the flow step (configs[2]) and the KD step (configs[3], distilTrain.py:156-185).
* the RCCL "overlap" schedule (bucketed all-reduces captured into the graph on a side stream
  as the backward completes each bucket) with a one-rank `nccl` process group (RCCL refuses
  two ranks on one device): the capture mechanics, bit-identical to the eager step."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batches(rank):
    import synthetic
    return [tuple(torch.from_numpy(a).cuda() for a in synthetic.ft3d_batch(1, 2048, seed=100 + 10 * s + rank))
            for s in range(3)]


def _worker(rank, port, out_dir, mode):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    from distill import graphed_flow_step, graphed_kd_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    model = PointConvBidirection().cuda()
    opt = make_optimizer(model, capturable=True)
    mine = _batches(rank)
    if mode == "kd":
        step = graphed_kd_step(_teacher(), model, opt, mine[0], warmup=1)
    else:
        step = graphed_flow_step(model, opt, mine[0], warmup=1)
    assert step.schedule == "serial"  # gloo collectives cannot be captured
    for i in (1, 2):
        step(*mine[i], next_batch=mine[i + 1] if i + 1 < len(mine) else None)
    torch.cuda.synchronize()
    torch.save({k: v.detach().cpu() for k, v in model.named_parameters()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _teacher():
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(5)
    return PointConvBidirection().cuda().eval()


def _loss(model, teacher, bt):
    import loss_functions
    if teacher is None:
        flows, fps1 = model(bt[0], bt[1], bt[0], bt[1])[:2]
        return loss_functions.multiScaleLoss(flows, bt[2], fps1)
    with torch.no_grad():
        t = teacher(bt[0], bt[1], bt[0], bt[1])
    o = model(bt[0], bt[1], bt[0], bt[1])
    return loss_functions.biDirection_loss_ht(o[0], o[5], o[6], o[1], o[2], bt[2], t[0], t[5],
                                              t[6], t[1], t[2], 0.3, 0.8, layer=3)


@pytest.mark.parametrize("mode", ["train", "kd"])
def test_graphed_step_world2_matches_averaged_eager(tmp_path, mode):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, str(tmp_path), mode)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0, p.exitcode
    p0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    p1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k
    # the same three steps eagerly in one process, gradients of the two ranks' batches averaged
    from distill import make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    model = PointConvBidirection().cuda().train()
    teacher = _teacher() if mode == "kd" else None
    opt = make_optimizer(model, capturable=True)
    b0, b1 = _batches(0), _batches(1)
    for i in range(3):
        opt.zero_grad(set_to_none=True)
        grads = []
        for bt in (b0[i], b1[i]):
            for p in model.parameters():
                p.grad = None
            _loss(model, teacher, bt).backward()
            grads.append([None if p.grad is None else p.grad.clone() for p in model.parameters()])
        for p, g0, g1 in zip(model.parameters(), *grads):
            p.grad = None if g0 is None else (g0 + g1) / 2
        opt.step()
    torch.cuda.synchronize()
    worst = 0.0
    for k, v in model.named_parameters():
        d = float((v.detach().cpu() - p0[k]).abs().max())
        scale = float(v.detach().abs().max()) + 1e-12
        worst = max(worst, d / scale)
    assert worst <= 1e-5, worst


def _nccl_worker(port, out_dir, mode):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from distill import graphed_flow_step, graphed_kd_step, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    model = PointConvBidirection().cuda()
    opt = make_optimizer(model, capturable=True)
    mine = _batches(0)
    if mode == "kd":
        step = graphed_kd_step(_teacher(), model, opt, mine[0], warmup=1, overlap=True)
    else:
        step = graphed_flow_step(model, opt, mine[0], warmup=1, overlap=True)
    assert step.schedule == "overlap" and len(step.buckets) > 1, (step.schedule, step.buckets)
    losses = [float(step(*mine[i], next_batch=mine[i + 1] if i + 1 < len(mine) else None))
              for i in (1, 2)]
    torch.cuda.synchronize()
    torch.save({"params": {k: v.detach().cpu() for k, v in model.named_parameters()},
                "losses": losses, "buckets": len(step.buckets)},
               os.path.join(out_dir, "nccl.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["train", "kd"])
def test_overlap_schedule_nccl_one_rank_equals_eager(tmp_path, mode):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), str(tmp_path), mode))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    got = torch.load(tmp_path / "nccl.pt", weights_only=True)
    from distill import FlowTrainStep, KDTrainStep, make_optimizer
    from models_bid_pointconv import PointConvBidirection
    torch.manual_seed(0)
    model = PointConvBidirection().cuda()
    opt = make_optimizer(model, capturable=True)
    eager = (KDTrainStep(_teacher(), model, opt) if mode == "kd" else FlowTrainStep(model, opt))
    b = _batches(0)
    eager(*b[0])
    losses = [float(eager(*b[i])) for i in (1, 2)]
    torch.cuda.synchronize()
    assert losses == got["losses"], (losses, got["losses"])
    for k, v in model.named_parameters():
        assert torch.equal(v.detach().cpu(), got["params"][k]), k
