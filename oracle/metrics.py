"""CPU oracle of the depth-evaluation metrics (test infrastructure only).

Restates, in numpy / torch CPU, what the reference computes per test batch:
  - src/test.py:105-118: clamp pred to [min_depth_eval, max_depth_eval]
    (then inf -> max, NaN -> min), keep min < gt < max inside the Eigen crop;
  - src/utils.py:45-66 compute_errors on the kept pixels;
  - src/GuideDepth/metrics.py:41-62 FastDepth Result.evaluate.
Pinned to tests/golden/golden_metrics.npz (captured by importing the
reference's own functions, tests/golden/make_golden.py).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def compute_errors(gt: np.ndarray, pred: np.ndarray) -> list[float]:
    """src/utils.py:45-66 (numpy, on the arrays' own dtype)."""
    thresh = np.maximum((gt / pred), (pred / gt))
    d1 = np.mean(thresh < 1.25)
    d2 = np.mean(thresh < 1.25 ** 2)
    d3 = np.mean(thresh < 1.25 ** 3)
    rms = np.sqrt(np.mean((gt - pred) ** 2))
    log_rms = np.sqrt(np.mean((np.log(gt) - np.log(pred)) ** 2))
    abs_rel = np.mean(np.abs(gt - pred) / gt)
    sq_rel = np.mean(((gt - pred) ** 2) / gt)
    err = np.log(pred) - np.log(gt)
    silog = np.sqrt(np.mean(err ** 2) - np.mean(err) ** 2) * 100
    log10 = np.mean(np.abs(np.log10(pred) - np.log10(gt)))
    return [float(v) for v in (silog, abs_rel, log10, rms, sq_rel, log_rms, d1, d2, d3)]


def eigen_crop(h: int, w: int) -> np.ndarray:
    """src/test.py:114-115."""
    return np.array([int(0.09375 * h), int(0.98125 * h),
                     int(0.0640625 * w), int(0.9390625 * w)]).astype(np.int32)


def batch_errors(gt_depth: np.ndarray, pred_depth: np.ndarray, min_depth_eval=1e-3,
                 max_depth_eval=80.0) -> list[float]:
    """src/test.py:105-118 for one batch of [n, h, w] maps (gt already DepthNorm'ed)."""
    pred = pred_depth.copy()
    pred[pred < min_depth_eval] = min_depth_eval
    pred[pred > max_depth_eval] = max_depth_eval
    pred[np.isinf(pred)] = max_depth_eval
    pred[np.isnan(pred)] = min_depth_eval
    mask = np.logical_and(gt_depth > min_depth_eval, gt_depth < max_depth_eval)
    crop = eigen_crop(gt_depth.shape[1], gt_depth.shape[2])
    crop_mask = np.zeros(mask.shape)
    crop_mask[:, crop[0]:crop[1], crop[2]:crop[3]] = 1
    mask = np.logical_and(mask, crop_mask)
    return compute_errors(gt_depth[mask], pred[mask])


def fastdepth_evaluate(output: torch.Tensor, target: torch.Tensor) -> dict:
    """src/GuideDepth/metrics.py:41-62 (torch CPU)."""
    abs_diff = (output - target).abs()
    mse = float((torch.pow(abs_diff, 2)).mean())
    l10 = lambda x: torch.log(x) / math.log(10)  # noqa: E731  (metrics.py:10-12)
    r = {"mse": mse, "rmse": math.sqrt(mse), "mae": float(abs_diff.mean()),
         "lg10": float((l10(output) - l10(target)).abs().mean()),
         "rmse_log": math.sqrt(torch.pow(l10(output) - l10(target), 2).mean()),
         "absrel": float((abs_diff / target).mean())}
    ratio = torch.max(output / target, target / output)
    for k, t in ((1, 1.25), (2, 1.25 ** 2), (3, 1.25 ** 3)):
        r[f"delta{k}"] = float((ratio < t).float().mean())
    inv = (1 / output - 1 / target).abs()
    r["irmse"] = math.sqrt((torch.pow(inv, 2)).mean())
    r["imae"] = float(inv.mean())
    return r
