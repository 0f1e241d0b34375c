"""ORACLE — TEST INFRASTRUCTURE ONLY.  Fixed random projections of parameter gradients.

A per-parameter gradient SUM hides elementwise errors that cancel; two projections onto
fixed N(0,1) vectors (seeded by the parameter name) do not.  The float64 reference run
(oracle/make_f64_fixture.py) stores sum_i g_i r_i and sum_i |g_i r_i| per parameter; the GPU
tests (tests/test_gpu_model.py) compute the same on the build's gradients.
"""
import zlib

import numpy as np


def projection_vectors(name, numel):
    """Two N(0,1) vectors per parameter, seeded by the parameter name (crc32)."""
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    return rng.standard_normal((2, numel))


def projection(name, grad):
    """-> ([g.r0, g.r1], [|g|.|r0|, |g|.|r1|]) in float64 (zeros for no gradient)."""
    if grad is None:
        return [0.0, 0.0], [0.0, 0.0]
    g = grad.detach().double().reshape(-1).cpu().numpy()
    r = projection_vectors(name, g.size)
    return list(r @ g), list(np.abs(r) @ np.abs(g))


def flow_layer_weight(name, shape):
    """The fixed output weighting of the flow-layer fixtures (make_fixtures.make_flow_layers;
    the GPU test regenerates it): loss = sum(out * weight)."""
    rng = np.random.default_rng([77, zlib.crc32(name.encode())])
    return rng.normal(size=shape).astype(np.float32)
