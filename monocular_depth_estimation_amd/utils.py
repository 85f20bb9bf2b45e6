"""Hot-path utilities of src/utils.py on MI355X.

DepthNorm (utils.py:7-8) runs on HIP kernels (device min/max reduction +
normalise, no host sync).  AverageMeter (:10-24) is host bookkeeping.
compute_errors (:45-66) and the per-batch evaluation of src/test.py:96-124
(clamp, range mask, Eigen crop) run on one HIP reduction (mde_eval_sums):
only the sixteen sums come back to the host.  colorize / hconcat_resize
(image logging) are not provided.
"""
from __future__ import annotations

import math

from .functional import depth_norm, eigen_crop, eval_sums


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


def errors_from_sums(s) -> list[float]:
    """[silog, abs_rel, log10, rms, sq_rel, log_rms, d1, d2, d3] (utils.py:45-66) from
    the mde_eval_sums sums; NaN when no pixel was selected (numpy's mean of [])."""
    s = [float(v) for v in (s.tolist() if hasattr(s, "tolist") else s)]
    n = s[0]
    if n == 0:
        return [math.nan] * 9
    d1, d2, d3 = s[1] / n, s[2] / n, s[3] / n
    rms = math.sqrt(s[4] / n)
    log_rms = math.sqrt(s[5] / n)
    abs_rel = s[6] / n
    sq_rel = s[7] / n
    mean_err = s[8] / n
    silog = math.sqrt(max(s[5] / n - mean_err * mean_err, 0.0)) * 100
    log10 = s[9] / n
    return [silog, abs_rel, log10, rms, sq_rel, log_rms, d1, d2, d3]


def compute_errors(gt, pred):
    """utils.py:45-66 on the GPU over the given (already selected) pixels.

    gt / pred: CUDA tensors of equal shape.  Returns the reference's list
    [silog, abs_rel, log10, rms, sq_rel, log_rms, d1, d2, d3] (Python floats).
    """
    return errors_from_sums(eval_sums(pred, gt))


def eval_batch_errors(gt_depth, pred_depth, min_depth_eval=1e-3, max_depth_eval=80.0,
                      crop=True):
    """One batch of src/test.py:96-118 on the GPU: pred clamped to
    [min_depth_eval, max_depth_eval] (NaN -> min), pixels with
    min_depth_eval < gt < max_depth_eval inside the Eigen crop, then
    compute_errors.  gt_depth / pred_depth: [n, 1, h, w] or [n, h, w] maps
    (gt already DepthNorm'ed, as test.py:91 does)."""
    h, w = gt_depth.shape[-2], gt_depth.shape[-1]
    c = eigen_crop(h, w) if crop else None
    return errors_from_sums(eval_sums(pred_depth, gt_depth, min_depth_eval, max_depth_eval,
                                      clamp_and_mask=True, crop=c))
