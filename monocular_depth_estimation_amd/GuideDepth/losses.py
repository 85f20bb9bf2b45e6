"""Depth_Loss of src/GuideDepth/losses.py on MI355X.

alpha * L1 + beta * clamp((1 - SSIM11) * 0.5, 0, 1) + gamma * grad, computed by
fused HIP kernels (11x11 separable Gaussian SSIM, image-gradient L1, L1);
backward recomputes on device from the forward's scalars.  Like the
reference it is a plain callable, not an nn.Module.
"""
from __future__ import annotations

from ..functional import depth_loss


class Depth_Loss:  # noqa: N801  (reference class name)
    def __init__(self, alpha, beta, gamma, maxDepth=10.0):  # noqa: N803
        self.alpha = alpha
        self.beta = beta
        self.gamma = gamma
        self.maxDepth = maxDepth
        self.last_parts = None

    def __call__(self, output, depth):
        loss, parts = depth_loss(output, depth, self.alpha, self.beta, self.gamma, self.maxDepth)
        self.last_parts = parts  # [loss, l1, l_ssim, l_grad, ssim_mean, count]
        return loss
