"""Depth losses of src/loss.py on MI355X (drop-in: same class names and call signatures).

SSIM (loss.py:57-88) runs as one fused HIP pass (functional.ssim3_l1) that
also yields its gradient; Silog_loss_variance (:116-129) is restated with
torch device ops — train.py computes it every step but never uses it
(train.py:98-100), so the training loop here skips it (see train.py).
"""
from __future__ import annotations

import torch
from torch import nn

from .functional import ssim3_l1


class SSIM(nn.Module):
    """Monodepth2 SSIM loss: mean(clamp((1 - SSIM(x, y)) / 2, 0, 1)) over a 3x3 window."""

    def __init__(self):
        super().__init__()
        self.C1 = 0.01 ** 2
        self.C2 = 0.03 ** 2

    def forward(self, x, y):
        return ssim3_l1(x, y, w_ssim=1.0, w_l1=0.0)[0]


class SSIML1(nn.Module):
    """w_ssim * SSIM(pred, t) + w_l1 * L1(pred, t) in one kernel (train.py:94-100 fused).

    With depth_norm=True the target is DepthNorm-ed inside the kernel
    (utils.py:7-8 / train.py:89), so the normalised target is never written.
    forward returns the scalar loss; `last_parts` holds [loss, ssim, l1] on device.
    """

    def __init__(self, w_ssim=1.0, w_l1=0.1, depth_norm=True):
        super().__init__()
        self.w_ssim, self.w_l1, self.depth_norm = float(w_ssim), float(w_l1), depth_norm
        self.last_parts = None

    def forward(self, pred, target):
        from .functional import minmax
        mm = minmax(target) if self.depth_norm else None
        loss, parts = ssim3_l1(pred, target, self.w_ssim, self.w_l1, target_minmax=mm)
        self.last_parts = parts
        return loss


class Silog_loss_variance(nn.Module):  # noqa: N801  (reference class name)
    """Scale-invariant log loss: 10 * sqrt(mean(d^2) - focus * mean(d)^2) over gt > 1e-3."""

    def __init__(self, variance_focus=0.85):
        super().__init__()
        self.variance_focus = variance_focus

    def forward(self, prediction, gt):
        """Same value as the reference's boolean-mask form (loss.py:121-129) but
        mask-multiplied: no data-dependent shape, so no host synchronisation
        and it can run inside a captured graph.  No valid pixel -> NaN, as the
        reference's mean over an empty selection."""
        valid = (gt > 1e-3).detach()
        n = valid.sum(dtype=torch.float32)  # a count: never rounded to bf16 under autocast
        safe_gt = torch.where(valid, gt, torch.ones_like(gt))
        d = torch.where(valid, torch.log(torch.clamp(prediction, min=1e-6)) - torch.log(safe_gt),
                        torch.zeros_like(prediction))
        mean_d = d.sum() / n
        return torch.sqrt((d * d).sum() / n - self.variance_focus * mean_d ** 2) * 10.0
