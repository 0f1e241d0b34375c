"""Scene-flow evaluation (reference: evaluate_bid_pointconv.py:27-172).

    python kd-pointcloud_amd/evaluate_bid_pointconv.py config_evaluate_bid_pointconv.yaml

Same configuration keys (dataset, data_root, num_points, batch_size, data_process,
allow_less_points, ckpt_dir + pretrain, workers), the same per-batch metrics averaged over
batches (the reference's AverageMeter with n = 1) and the same report line.  MI355X-first:
batches arrive in HBM one step ahead (datasets.DeviceLoader), the forward runs under
inference mode, and every metric -- multiScaleLoss, EPE3D, ACC3DS/R, outliers, EPE2D,
ACC2D -- is computed on the device and accumulated there; the host reads the totals once,
at the end, instead of the reference's five `.cpu()` copies and NumPy metrics per batch.
Checkpoints load with torch.load(weights_only=True)."""
import os
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import datasets  # noqa: E402
import loss_functions  # noqa: E402
import transforms  # noqa: E402
from evaluation_utils import evaluate_2d, evaluate_3d  # noqa: E402
from utils import geometry  # noqa: E402

METRICS = ("loss", "epe", "EPE3D", "ACC3DS", "ACC3DR", "Outliers3D", "EPE2D", "ACC2D")


@torch.inference_mode()
def evaluate(model, loader, calib_dir=None, loss_fn=None):
    """Per-batch metrics of `model` over `loader` (yielding (pos1, pos2, norm1, norm2, flow,
    paths)), averaged over batches.  loss / epe are the reference's sample-weighted running
    means (total_loss / total_seen); the others are means of per-batch values.  Returns a
    dict of Python floats (one device-to-host copy)."""
    loss_fn = loss_fn or loss_functions.multiScaleLoss
    model.eval()
    acc = None
    nb = 0
    seen = 0
    for pos1, pos2, norm1, norm2, flow, paths in loader:
        out = model(pos1, pos2, norm1, norm2)
        pred_flows, fps_idx = out[0], out[1]
        b = pos1.shape[0]
        full = pred_flows[0].permute(0, 2, 1)
        loss = loss_fn(pred_flows, flow, fps_idx)
        epe = torch.linalg.vector_norm(full - flow, dim=2).mean()
        m3 = evaluate_3d(full, flow)
        fp, fg = geometry.get_batch_2d_flow(pos1, pos1 + flow, pos1 + full, paths, calib_dir)
        m2 = evaluate_2d(fp, fg)
        row = torch.stack([v.reshape(()).double() for v in
                           (loss * b, epe * b, *m3, *m2)])
        acc = row if acc is None else acc + row
        nb += 1
        seen += b
    if acc is None:
        raise RuntimeError("evaluate: empty loader")
    vals = acc.cpu().tolist()
    res = {k: v / (seen if k in ("loss", "epe") else nb) for k, v in zip(METRICS, vals)}
    res["batches"], res["samples"] = nb, seen
    return res


def format_result(r):
    """The reference's report line (evaluate_bid_pointconv.py:150-166)."""
    return (" * EPE3D {:.4f}\tACC3DS {:.4f}\tACC3DR {:.4f}\tOutliers3D {:.4f}\tEPE2D {:.4f}\t"
            "ACC2D {:.4f}").format(r["EPE3D"], r["ACC3DS"], r["ACC3DR"], r["Outliers3D"],
                                   r["EPE2D"], r["ACC2D"])


def _ns(d):
    return types.SimpleNamespace(**{k: _ns(v) if isinstance(v, dict) and k not in
                                    ("data_process", "aug_together", "aug_pc2") else v
                                    for k, v in d.items()})


def make_val_dataset(args):
    kw = dict(train=False,
              transform=transforms.ProcessData(args.data_process, args.num_points,
                                               getattr(args, "allow_less_points", False)),
              num_points=args.num_points, data_root=args.data_root)
    return getattr(datasets, args.dataset)(**kw)


def main(config_path):
    import yaml
    with open(config_path) as fd:
        args = _ns(yaml.safe_load(fd))
    from models_bid_lighttoken_res import PointConvBidirection
    dev = torch.device("cuda", 0)
    model = PointConvBidirection()
    pretrain = getattr(args, "pretrain", "") or ""
    ckpt = os.path.join(getattr(args, "ckpt_dir", "") or "", pretrain)
    if pretrain:
        if not os.path.isfile(ckpt):  # the reference's torch.load raises here too
            raise FileNotFoundError(f"checkpoint {ckpt!r} (ckpt_dir + pretrain) does not exist")
        model.load_state_dict(torch.load(ckpt, map_location="cpu", weights_only=True))
        print("load model %s" % ckpt)
    elif getattr(args, "allow_random_init", False):
        print("no pretrain given (allow_random_init): evaluating random-init weights")
    else:
        raise ValueError("no checkpoint: set `pretrain` (with `ckpt_dir`), or "
                         "`allow_random_init: true` to evaluate random-init weights")
    model.to(dev)
    loader = datasets.DeviceLoader(make_val_dataset(args), args.batch_size, dev,
                                   num_workers=getattr(args, "workers", 0))
    r = evaluate(model, loader, calib_dir=getattr(args, "calib_dir", None))
    print("Evaluate mean loss: %f mean epe: %f" % (r["loss"], r["epe"]))
    print(format_result(r))
    return r


if __name__ == "__main__":
    main(sys.argv[1])
