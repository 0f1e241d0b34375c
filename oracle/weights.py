"""ORACLE / TEST INFRASTRUCTURE: deterministic synthetic weights.

The reference's pretrained checkpoints are missing (.MISSING_LARGE_BLOBS), so fixtures and
parity tests use weights generated from the state_dict KEY NAMES alone:
tensor(key) ~ numpy default_rng([seed, crc32(key)]), scaled like PyTorch's default init
(U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for conv/linear weights and biases), BN affine/statistics
drawn near identity, the unused cost-volume biases ~ N(0,1).  Any module tree with the
reference's key names (reference, oracle/torch_model.py, kd-pointcloud_amd) gets identical
tensors, so only inputs/outputs need to be committed.
"""
import zlib

import numpy as np
import torch


def _rng(seed, key):
    return np.random.default_rng([seed, zlib.crc32(key.encode())])


def synthetic_state_dict(template, seed=0):
    """template: a state_dict (only key names, shapes and dtypes are used)."""
    out = {}
    for key, ref in template.items():
        shape = tuple(ref.shape)
        rng = _rng(seed, key)
        leaf = key.rsplit(".", 1)[-1]
        is_bn = ("bn" in key.split(".")[-2]) if "." in key else False
        if ref.dtype in (torch.int64, torch.int32):
            out[key] = torch.zeros(shape, dtype=ref.dtype)
            continue
        if leaf == "running_mean":
            v = rng.uniform(-0.1, 0.1, shape)
        elif leaf == "running_var":
            v = rng.uniform(0.5, 1.5, shape)
        elif is_bn and leaf == "weight":
            v = rng.uniform(0.5, 1.5, shape)
        elif is_bn and leaf == "bias":
            v = rng.uniform(-0.1, 0.1, shape)
        elif leaf in ("bias1", "bias2", "bias") and len(shape) == 4:
            v = rng.normal(0.0, 1.0, shape)
        elif leaf == "weight" and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            b = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-b, b, shape)
        elif leaf == "bias":
            wkey = key[: -len("bias")] + "weight"
            w = template.get(wkey)
            fan_in = int(np.prod(tuple(w.shape)[1:])) if w is not None and w.dim() >= 2 else shape[0]
            b = 1.0 / np.sqrt(max(fan_in, 1))
            v = rng.uniform(-b, b, shape)
        else:
            v = rng.normal(0.0, 0.1, shape)
        out[key] = torch.from_numpy(np.asarray(v, dtype=np.float32))
    return out


def load_synthetic(module, seed=0):
    module.load_state_dict(synthetic_state_dict(module.state_dict(), seed))
    return module
