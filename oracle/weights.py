"""Deterministic parameter fill shared by the golden-capture script and tests.

The fixtures do not store weights: every floating state_dict entry is filled
by a formula of its NAME and SHAPE only (numpy PCG64 seeded by crc32(name)),
so the reference module (at capture time), the oracle and the HIP model all
receive identical weights.  Integer buffers (num_batches_tracked,
relative_position_index) are left alone.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def tensor_for(name: str, shape) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    z = rng.standard_normal(shape).astype(np.float32)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "running_var":
        return (1.0 + 0.25 * np.abs(z)).astype(np.float32)
    if leaf == "running_mean":
        return (0.1 * z).astype(np.float32)
    if "relative_position_bias_table" in name:
        return (0.02 * z).astype(np.float32)
    if len(shape) <= 1:
        if leaf == "weight":  # BatchNorm / LayerNorm affine scale
            return (1.0 + 0.1 * z).astype(np.float32)
        return (0.05 * z).astype(np.float32)  # biases
    fan_in = int(np.prod(shape[1:]))
    return (z * np.sqrt(2.0 / fan_in)).astype(np.float32)


@torch.no_grad()
def fill_(module: torch.nn.Module) -> torch.nn.Module:
    for name, t in module.state_dict().items():
        if not t.is_floating_point():
            continue
        t.copy_(torch.from_numpy(tensor_for(name, t.shape)).to(t.dtype))
    return module


def seeded(shape, seed: int, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """Uniform [lo, hi) fp32 test input from numpy PCG64(seed)."""
    rng = np.random.default_rng(seed)
    return (lo + (hi - lo) * rng.random(tuple(shape))).astype(np.float32)
