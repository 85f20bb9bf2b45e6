"""Guided-upsampling and squeeze-excitation blocks on MI355X.

Drop-in for src/GuideDepth/model/modules.py: same constructors, forward
signatures and state_dict keys.  Hot ops on HIP kernels:
  * cat([x, y], 1) + SELayer (:90, :21-25)  -> functional.se_cat (one fused op,
    the concatenation is never materialised); in training (fp32, or bf16 under
    autocast) together with
    the two branches' last BatchNorm + ReLU (:49, :59) -> nn.se_bn_cat, which
    reads the 1x1 convs' raw outputs and writes only the SE output;
  * reduce(residual + depth) (:100)          -> functional.skip_reduce.
Convolutions stay on PyTorch-ROCm (MIOpen) without their bias; conv bias +
BatchNorm + ReLU run as one fused HIP pass (nn.py run_sequential).
"""
from __future__ import annotations

from torch import nn

from ...functional import se_cat, skip_reduce
from ...nn import (BatchNorm2d, batch_norm_act, run_sequential, run_sequential_raw, se_bn_cat,
                   skip_reduce_bn, skip_reduce_bn_ok)

# Guided_Upsampling_Block (training; fp32, or bf16 storage under autocast): run the branches' last BN + ReLU,
# the concatenation and SE as one fused op (nn.se_bn_cat), and the comb_conv's
# last BN + ReLU inside the skip fusion's operand load (nn.skip_reduce_bn).
FUSE_BN = True


class SELayer(nn.Module):
    """Channel attention: mean_hw -> Linear -> ReLU -> Linear -> Sigmoid -> scale.

    reference modules.py:5-25 (both Linear layers bias-free).
    """

    def __init__(self, channel, reduction=16):
        super().__init__()
        hidden = channel // reduction
        self.fc = nn.Sequential(nn.Linear(channel, hidden, bias=False), nn.ReLU(inplace=True),
                                nn.Linear(hidden, channel, bias=False), nn.Sigmoid())

    def forward(self, x):
        return se_cat(x, None, self.fc[0].weight, self.fc[2].weight)

    def forward_cat(self, x, y):
        """SELayer(torch.cat([x, y], 1)) without materialising the concatenation."""
        return se_cat(x, y, self.fc[0].weight, self.fc[2].weight)


def _conv_bn_relu(cin, cout, k):
    """conv -> BN+ReLU fused on the HIP kernel (Identity keeps the ReLU's Sequential slot)."""
    return [nn.Conv2d(cin, cout, kernel_size=k, padding=k // 2), BatchNorm2d(cout, act="relu"),
            nn.Identity()]


class Guided_Upsampling_Block(nn.Module):  # noqa: N801  (reference class name)
    """Refines an upsampled depth feature map with the RGB guide (modules.py:29-100).

    feature_conv(depth) and guide_conv(guide) each: kxk conv -> BN -> ReLU ->
    1x1 conv (E -> E/2) -> BN -> ReLU.  Their concatenation goes through SE,
    comb_conv (kxk conv -> BN -> ReLU -> 1x1 -> BN -> ReLU), and the result
    plus `depth` goes through the 1x1 `reduce` conv.
    """

    def __init__(self, in_features, expand_features, out_features, kernel_size=3,
                 channel_attention=True, guidance_type="full", guide_features=3):
        super().__init__()
        self.channel_attention = channel_attention
        self.guidance_type = guidance_type
        self.guide_features = guide_features
        self.in_features = in_features
        e, k = expand_features, kernel_size
        self.feature_conv = nn.Sequential(*_conv_bn_relu(in_features, e, k),
                                          *_conv_bn_relu(e, e // 2, 1))
        if guidance_type == "full":
            self.guide_conv = nn.Sequential(*_conv_bn_relu(guide_features, e, k),
                                            *_conv_bn_relu(e, e // 2, 1))
            comb_features = (e // 2) * 2
        elif guidance_type == "raw":
            comb_features = e // 2 + guide_features
        else:
            comb_features = e // 2
        self.comb_conv = nn.Sequential(*_conv_bn_relu(comb_features, e, k),
                                       *_conv_bn_relu(e, in_features, 1))
        self.reduce = nn.Conv2d(in_features, out_features, kernel_size=1)
        if channel_attention:
            self.SE_block = SELayer(comb_features, reduction=1)

    def forward(self, guide, depth):
        if FUSE_BN and self.channel_attention and self.guidance_type == "full":
            # the branches' last BN + ReLU, the concatenation and SE as one op
            ra = run_sequential_raw(self.feature_conv, depth)
            rb = run_sequential_raw(self.guide_conv, guide) if ra is not None else None
            if rb is not None:
                xy = se_bn_cat(ra[0], rb[0], ra[2], rb[2], ra[3], rb[3],
                               self.SE_block.fc[0].weight, self.SE_block.fc[2].weight,
                               ra[1], rb[1])
                return self._comb_reduce(xy, depth)
            if ra is not None:  # finish the feature branch unfused
                x = batch_norm_act(ra[0], ra[2], ra[2].act, None, ra[3], ra[1])
                second = run_sequential(self.guide_conv, guide)
                xy = self.SE_block.forward_cat(x, second)
                return self._comb_reduce(xy, depth)
        x = run_sequential(self.feature_conv, depth)
        if self.guidance_type == "full":
            second = run_sequential(self.guide_conv, guide)
        elif self.guidance_type == "raw":
            second = guide
        else:
            second = None
        if self.channel_attention:
            xy = self.SE_block.forward_cat(x, second) if second is not None else self.SE_block(x)
        else:
            xy = x if second is None else _cat(x, second)
        if FUSE_BN:
            return self._comb_reduce(xy, depth)
        return skip_reduce(run_sequential(self.comb_conv, xy), depth, self.reduce.weight,
                           self.reduce.bias)

    def _comb_reduce(self, xy, depth):
        """comb_conv + reduce(residual + depth) with the comb_conv's last BN +
        ReLU applied inside the skip kernel's operand load (nn.skip_reduce_bn)
        where that runs (training, fp32 or bf16, supported shapes)."""
        rc = run_sequential_raw(self.comb_conv, xy)
        if rc is None:
            return skip_reduce(run_sequential(self.comb_conv, xy), depth, self.reduce.weight,
                               self.reduce.bias)
        y2, st2, bn2, pb2 = rc
        if skip_reduce_bn_ok(y2, self.reduce.out_channels):
            return skip_reduce_bn(y2, bn2, pb2, depth, self.reduce.weight, self.reduce.bias, st2)
        x = batch_norm_act(y2, bn2, bn2.act, None, pb2, st2)
        return skip_reduce(x, depth, self.reduce.weight, self.reduce.bias)


def _cat(x, y):
    import torch
    return torch.cat([x, y], dim=1)
