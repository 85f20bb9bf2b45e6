"""MobileNetV3-Large feature extractor on MI355X (restates torchvision's published architecture).

The reference calls torchvision.models.mobilenet_v3_large(pretrained=True)
(src/model_mobileV3_large_newCRFs.py:165) and runs `.features` module by
module (:178-182).  torchvision is absent from this stack, so this module
rebuilds the same network — 16-channel hardswish stem, the 15 inverted
residual blocks of the Large table (expand 1x1 -> depthwise k3/k5 s1/s2 ->
[squeeze-excitation, hardsigmoid gate] -> project 1x1, residual when stride 1
and in == out), 960-channel 1x1 head, BatchNorm eps 1e-3 momentum 0.01 — with
torchvision's module tree, so state_dict keys (`features.3.block.1.0.weight`,
...) match a torchvision checkpoint.  Parity is UNPINNED: no torchvision
oracle can run here; the feature shapes are pinned by the reference's own
comment (model_mobileV3_large_newCRFs.py:94-111) and its decoder's
in_channels [24, 40, 112, 160, 960] (:71).

Every BatchNorm (with its ReLU / Hardswish) runs fused on the HIP BN kernel;
the depthwise convolutions + BN + activation run on the HIP depthwise kernel;
the 1x1 expand / project convs on the NCHW HIP 1x1 kernels (conv1x1.hip, the
channel counts that are not multiples of 32 padded in-kernel).
"""
from __future__ import annotations

from functools import partial

import torch
from torch import nn

from .nn import BatchNorm2d, Conv2d, batch_norm_act, depthwise_conv_bn_act, se_hardsigmoid


def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


_ACT = {"RE": "relu", "HS": "hardswish", None: "none"}


class Conv2dNormActivation(nn.Sequential):
    """conv (no bias) -> BatchNorm -> activation; keys `0.weight`, `1.*` like torchvision."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1, act="relu",
                 norm_layer=partial(BatchNorm2d, eps=0.001, momentum=0.01)):
        pad = (kernel_size - 1) // 2
        # nn.py's Conv2d: the 1x1 convs on the NCHW HIP kernels (conv1x1.hip,
        # channel counts padded to 32), the rest as the stock module
        super().__init__(Conv2d(cin, cout, kernel_size, stride, pad, groups=groups, bias=False),
                         norm_layer(cout, act=act), nn.Identity())
        self.act = act

    def forward(self, x, residual=None):
        conv, bn = self[0], self[1]
        if conv.groups == conv.in_channels == conv.out_channels and conv.groups > 1:
            return depthwise_conv_bn_act(x, conv, bn, bn.act)
        return batch_norm_act(conv(x), bn, bn.act, residual)


class SqueezeExcitation(nn.Module):
    """avgpool -> fc1 (1x1, bias) -> ReLU -> fc2 (1x1, bias) -> hardsigmoid -> scale (torchvision.ops)."""

    def __init__(self, input_channels, squeeze_channels):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(input_channels, squeeze_channels, 1)
        self.fc2 = nn.Conv2d(squeeze_channels, input_channels, 1)
        self.activation = nn.ReLU()
        self.scale_activation = nn.Hardsigmoid()

    def forward(self, x):
        return se_hardsigmoid(x, self.fc1, self.fc2)


class InvertedResidual(nn.Module):
    def __init__(self, cin, kernel, expanded, cout, use_se, act, stride):
        super().__init__()
        a = _ACT[act]
        layers = []
        if expanded != cin:
            layers.append(Conv2dNormActivation(cin, expanded, 1, act=a))
        layers.append(Conv2dNormActivation(expanded, expanded, kernel, stride, groups=expanded, act=a))
        if use_se:
            layers.append(SqueezeExcitation(expanded, _make_divisible(expanded // 4, 8)))
        layers.append(Conv2dNormActivation(expanded, cout, 1, act="none"))
        self.block = nn.Sequential(*layers)
        self.out_channels = cout
        self._is_cn = stride > 1
        self.use_res_connect = stride == 1 and cin == cout

    def forward(self, x):
        mods = list(self.block)
        y = x
        for m in mods[:-1]:
            y = m(y)
        # the residual add runs inside the projection's BN pass
        return mods[-1](y, residual=x if self.use_res_connect else None)


# (input, kernel, expanded, output, use_se, activation, stride) — the Large table
LARGE = [
    (16, 3, 16, 16, False, "RE", 1), (16, 3, 64, 24, False, "RE", 2), (24, 3, 72, 24, False, "RE", 1),
    (24, 5, 72, 40, True, "RE", 2), (40, 5, 120, 40, True, "RE", 1), (40, 5, 120, 40, True, "RE", 1),
    (40, 3, 240, 80, False, "HS", 2), (80, 3, 200, 80, False, "HS", 1), (80, 3, 184, 80, False, "HS", 1),
    (80, 3, 184, 80, False, "HS", 1), (80, 3, 480, 112, True, "HS", 1), (112, 3, 672, 112, True, "HS", 1),
    (112, 5, 672, 160, True, "HS", 2), (160, 5, 960, 160, True, "HS", 1), (160, 5, 960, 160, True, "HS", 1),
]


class MobileNetV3(nn.Module):
    def __init__(self, num_classes=1000, last_channel=1280, dropout=0.2):
        super().__init__()
        layers = [Conv2dNormActivation(3, 16, 3, 2, act="hardswish")]
        layers += [InvertedResidual(*cfg) for cfg in LARGE]
        layers.append(Conv2dNormActivation(160, 960, 1, act="hardswish"))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Linear(960, last_channel), nn.Hardswish(inplace=True),
                                        nn.Dropout(p=dropout, inplace=True),
                                        nn.Linear(last_channel, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


def mobilenet_v3_large(num_classes=1000):
    return MobileNetV3(num_classes=num_classes)
