"""CPU restatement of the hot-path ops (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Everything is written out from the reference's semantics with torch CPU
tensor algebra (gathers, shifted slices, sums) so autograd supplies the
gradients; nothing here calls F.interpolate / avg_pool2d / conv2d for the
restated ops.  Resize index tables are built in numpy float32 the way ATen's
upsample kernels compute them (area_pixel_compute_source_index,
nearest_neighbor_compute_source_index).
"""
from __future__ import annotations

import math

import numpy as np
import torch

# ------------------------------------------------------------------ resizes


def resize_plan(hi: int, wi: int, size=None, scale_factor=None, align_corners=False):
    """(ho, wo, scale_h, scale_w) as F.interpolate hands them to ATen.

    size -> scale = in/out (fp32); scale_factor s -> out = floor(in*s),
    scale = 1/s; align_corners -> (in-1)/(out-1).
    """
    if size is not None:
        ho, wo = (size, size) if isinstance(size, int) else (int(size[0]), int(size[1]))
        sh = np.float32(hi) / np.float32(ho)
        sw = np.float32(wi) / np.float32(wo)
    else:
        sf = (scale_factor, scale_factor) if isinstance(scale_factor, (int, float)) else scale_factor
        ho, wo = int(math.floor(hi * float(sf[0]))), int(math.floor(wi * float(sf[1])))
        sh, sw = np.float32(1.0 / float(sf[0])), np.float32(1.0 / float(sf[1]))
    if align_corners:
        sh = np.float32(hi - 1) / np.float32(ho - 1) if ho > 1 else np.float32(0)
        sw = np.float32(wi - 1) / np.float32(wo - 1) if wo > 1 else np.float32(0)
    return ho, wo, np.float32(sh), np.float32(sw)


def linear_table(in_size: int, out_size: int, scale, align_corners: bool):
    """i0, i1, l0, l1 per output index (ATen upsample_bilinear2d, one axis)."""
    s = np.float32(scale)
    o = np.arange(out_size, dtype=np.float32)
    if align_corners:
        src = s * o
    else:
        src = s * (o + np.float32(0.5)) - np.float32(0.5)
        src = np.maximum(src, np.float32(0.0))
    i0 = np.minimum(np.floor(src).astype(np.int64), in_size - 1)
    i1 = np.minimum(i0 + 1, in_size - 1)
    l1 = np.clip(src - i0.astype(np.float32), 0.0, 1.0).astype(np.float32)
    l0 = (np.float32(1.0) - l1).astype(np.float32)
    return i0, i1, l0, l1


def bilinear(x: torch.Tensor, size=None, scale_factor=None, align_corners=False):
    """F.interpolate(x, size|scale_factor, mode='bilinear', align_corners)."""
    hi, wi = x.shape[-2:]
    ho, wo, sh, sw = resize_plan(hi, wi, size, scale_factor, align_corners)
    h0, h1, a0, a1 = linear_table(hi, ho, sh, align_corners)
    w0, w1, b0, b1 = linear_table(wi, wo, sw, align_corners)
    t = lambda v: torch.from_numpy(v)
    r0 = x.index_select(2, t(h0))
    r1 = x.index_select(2, t(h1))
    bw0, bw1 = t(b0).view(1, 1, 1, -1), t(b1).view(1, 1, 1, -1)
    top = bw0 * r0.index_select(3, t(w0)) + bw1 * r0.index_select(3, t(w1))
    bot = bw0 * r1.index_select(3, t(w0)) + bw1 * r1.index_select(3, t(w1))
    return t(a0).view(1, 1, -1, 1) * top + t(a1).view(1, 1, -1, 1) * bot


def nearest_table(in_size: int, out_size: int, scale):
    o = np.arange(out_size, dtype=np.float32)
    return np.minimum(np.floor(o * np.float32(scale)).astype(np.int64), in_size - 1)


def nearest(x: torch.Tensor, size=None, scale_factor=None):
    """F.interpolate(x, size|scale_factor) (mode='nearest')."""
    hi, wi = x.shape[-2:]
    ho, wo, sh, sw = resize_plan(hi, wi, size, scale_factor, False)
    rows = torch.from_numpy(nearest_table(hi, ho, sh))
    cols = torch.from_numpy(nearest_table(wi, wo, sw))
    return x.index_select(2, rows).index_select(3, cols)


# ------------------------------------------------------- SE and skip fusion


def se(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """SELayer.forward (src/GuideDepth/model/modules.py:21-25)."""
    m = x.mean(dim=(2, 3))
    s = torch.sigmoid(torch.relu(m @ w1.t()) @ w2.t())
    return x * s[:, :, None, None]


def skip_reduce(r, d, weight, bias):
    """reduce(residual + depth) (modules.py:100) with a 1x1 conv weight [o, c, 1, 1]."""
    s = r + d
    return torch.einsum("oc,nchw->nohw", weight.reshape(weight.shape[0], -1), s) + bias.view(1, -1, 1, 1)


# ------------------------------------------------------------------ losses


def depth_norm(d: torch.Tensor) -> torch.Tensor:
    """DepthNorm (src/utils.py:7-8)."""
    return (d - d.min()) / (d.max() - d.min())


def _reflect1(z: torch.Tensor) -> torch.Tensor:
    """ReflectionPad2d(1) written as index gathers."""
    h, w = z.shape[-2:]
    rows = torch.tensor([1] + list(range(h)) + [h - 2])
    cols = torch.tensor([1] + list(range(w)) + [w - 2])
    return z.index_select(2, rows).index_select(3, cols)


def _box3(zp: torch.Tensor, h: int, w: int) -> torch.Tensor:
    acc = None
    for a in range(3):
        for b in range(3):
            v = zp[:, :, a:a + h, b:b + w]
            acc = v if acc is None else acc + v
    return acc / 9.0


def ssim3(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """loss.SSIM()(x, y) (src/loss.py:57-88)."""
    h, w = x.shape[-2:]
    xp, yp = _reflect1(x), _reflect1(y)
    mx, my = _box3(xp, h, w), _box3(yp, h, w)
    sx = _box3(xp * xp, h, w) - mx * mx
    sy = _box3(yp * yp, h, w) - my * my
    sxy = _box3(xp * yp, h, w) - mx * my
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    n = (2 * mx * my + c1) * (2 * sxy + c2)
    dd = (mx * mx + my * my + c1) * (sx + sy + c2)
    return torch.clamp((1 - n / dd) / 2, 0, 1).mean()


def l1(x, y):
    """nn.L1Loss() (src/train.py:53)."""
    return (x - y).abs().mean()


def train_loss(pred, depth):
    """The train.py objective: DepthNorm target, 1.0*SSIM + 0.1*L1 (train.py:89-100)."""
    t = depth_norm(depth)
    return 1.0 * ssim3(pred, t) + 0.1 * l1(pred, t)


def silog(pred, gt, variance_focus=0.85):
    """Silog_loss_variance (src/loss.py:116-129)."""
    mask = gt > 1e-3
    p = torch.clamp(pred, min=1e-6)[mask]
    g = gt[mask]
    d = torch.log(p) - torch.log(g)
    return torch.sqrt((d ** 2).mean() - variance_focus * d.mean() ** 2) * 10.0


def gaussian_1d(k: int, sigma: float = 1.5) -> torch.Tensor:
    """Depth_Loss.gaussian (src/GuideDepth/losses.py:125-127)."""
    g = torch.tensor([math.exp(-(x - k // 2) ** 2 / float(2 * sigma ** 2)) for x in range(k)],
                     dtype=torch.float32)
    return g / g.sum()


def _window_sum(zp: torch.Tensor, win: torch.Tensor, ho: int, wo: int) -> torch.Tensor:
    k = win.shape[0]
    acc = None
    for a in range(k):
        for b in range(k):
            v = win[a, b] * zp[:, :, a:a + ho, b:b + wo]
            acc = v if acc is None else acc + v
    return acc


def ssim11(img1, img2, val_range):
    """Depth_Loss.ssim with its defaults (losses.py:41-79): mean SSIM map."""
    _, c, h, w = img1.shape
    k = min(11, h, w)
    g = gaussian_1d(k).unsqueeze(1)
    win = (g @ g.t()).float()
    pad = 11 // 2
    ho, wo = h + 2 * pad - k + 1, w + 2 * pad - k + 1
    zp = lambda z: torch.nn.functional.pad(z, (pad, pad, pad, pad))
    p1, p2 = zp(img1), zp(img2)
    mu1, mu2 = _window_sum(p1, win, ho, wo), _window_sum(p2, win, ho, wo)
    s11 = _window_sum(p1 * p1, win, ho, wo) - mu1 * mu1
    s22 = _window_sum(p2 * p2, win, ho, wo) - mu2 * mu2
    s12 = _window_sum(p1 * p2, win, ho, wo) - mu1 * mu2
    c1, c2 = (0.01 * val_range) ** 2, (0.03 * val_range) ** 2
    v1 = 2.0 * s12 + c2
    v2 = s11 + s22 + c2
    return (((2 * mu1 * mu2 + c1) * v1) / ((mu1 * mu1 + mu2 * mu2 + c1) * v2)).mean()


def image_gradients(x):
    """Depth_Loss.gradient (losses.py:95-115): forward differences, last col/row 0."""
    dx = torch.zeros_like(x)
    dy = torch.zeros_like(x)
    dx = torch.cat([x[..., 1:] - x[..., :-1], torch.zeros_like(x[..., :1])], dim=-1)
    dy = torch.cat([x[..., 1:, :] - x[..., :-1, :], torch.zeros_like(x[..., :1, :])], dim=-2)
    return dx, dy


def depth_loss(output, depth, alpha, beta, gamma, max_depth=10.0):
    """Depth_Loss(alpha, beta, gamma, maxDepth)(output, depth) (losses.py:15-38)."""
    if beta == 0 and gamma == 0:
        m = depth > 0.0
        return (output[m] - depth[m]).abs().mean()
    l_depth = l1(output, depth)
    l_ssim = torch.clamp((1 - ssim11(output, depth, max_depth)) * 0.5, 0, 1)
    pdx, pdy = image_gradients(output)
    gdx, gdy = image_gradients(depth)
    l_grad = ((gdx - pdx).abs() + (gdy - pdy).abs()).mean()
    return alpha * l_depth + beta * l_ssim + gamma * l_grad
