"""Scene-flow metrics (reference: evaluation_utils.py:18-50, HPLFlowNet's definitions).

Each function accepts NumPy arrays -- then it computes exactly what the reference computes
(float32 norms and means, float64 fractions; `np.float` of the reference is float64) -- or
torch tensors, in which case it stays on the tensors' device and returns 0-d tensors, so an
evaluation loop on the GPU never synchronises per batch (evaluate_bid_pointconv.evaluate)."""
import numpy as np
import torch


def _norm(x):
    return torch.linalg.vector_norm(x, dim=-1) if torch.is_tensor(x) else np.linalg.norm(x, axis=-1)


def _frac(mask):
    return mask.double().mean() if torch.is_tensor(mask) else mask.astype(np.float64).mean()


def _or(a, b):
    return torch.logical_or(a, b) if torch.is_tensor(a) else np.logical_or(a, b)


def evaluate_3d(sf_pred, sf_gt):
    """sf_pred, sf_gt (..., N, 3) -> (EPE3D, ACC3D strict, ACC3D relax, outliers):
    EPE3D = mean |gt - pred|; strict: EPE < 0.05 or relative < 5 %; relax: < 0.1 or < 10 %;
    outlier: EPE > 0.3 or relative > 10 % (relative = EPE / (|gt| + 1e-4))."""
    l2 = _norm(sf_gt - sf_pred)
    epe = l2.mean()
    rel = l2 / (_norm(sf_gt) + 1e-4)
    strict = _frac(_or(l2 < 0.05, rel < 0.05))
    relax = _frac(_or(l2 < 0.1, rel < 0.1))
    outlier = _frac(_or(l2 > 0.3, rel > 0.1))
    return epe, strict, relax, outlier


def evaluate_2d(flow_pred, flow_gt):
    """flow_pred, flow_gt (..., N, 2) -> (EPE2D, ACC2D: EPE < 3 px or relative < 5 %)."""
    epe = _norm(flow_gt - flow_pred)
    rel = epe / (_norm(flow_gt) + 1e-5)
    return epe.mean(), _frac(_or(epe < 3.0, rel < 0.05))
