"""Hot-path utilities of src/utils.py on MI355X.

DepthNorm (utils.py:7-8) runs on HIP kernels (device min/max reduction +
normalise, no host sync).  AverageMeter (:10-24) is host bookkeeping.
compute_errors / colorize (evaluation and logging) are outside the training
hot path and are not provided here.
"""
from __future__ import annotations

from .functional import depth_norm


def DepthNorm(depth):  # noqa: N802  (reference name)
    """(depth - depth.min()) / (depth.max() - depth.min()), batch-global."""
    return depth_norm(depth)


class AverageMeter:
    """Running value / sum / count / average (utils.py:10-24)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
