"""CPU restatement of MobileNetV3-Large + the NewCRF PTModel (TEST INFRASTRUCTURE ONLY).

The reference takes its encoder from torchvision.models.mobilenet_v3_large
(src/model_mobileV3_large_newCRFs.py:165,178-182).  torchvision is not in
this image, so this file restates torchvision's published Large table with
stock torch.nn layers (Conv2d, BatchNorm2d eps 1e-3 momentum 0.01, ReLU,
Hardswish, Hardsigmoid); its module tree gives torchvision's state_dict keys.
PARITY UNPINNED: no reference output exists for the encoder; only the
feature shapes/channels of the reference comment (:94-111) and the decoder's
in_channels (:71) pin it.  The decoder half (oracle/newcrf.Decoder) IS
pinned by the reference goldens (tests/golden/golden_newcrf.npz).
"""
from __future__ import annotations

import torch
from torch import nn

from .newcrf import Decoder


def _div8(v):
    nv = max(8, int(v + 4) // 8 * 8)
    return nv + 8 if nv < 0.9 * v else nv


def _cna(cin, cout, k, stride=1, groups=1, act=None):
    mods = [nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
            nn.BatchNorm2d(cout, eps=0.001, momentum=0.01)]
    if act is not None:
        mods.append(act())
    return nn.Sequential(*mods)


class SE(nn.Module):
    def __init__(self, c, s):
        super().__init__()
        self.fc1 = nn.Conv2d(c, s, 1)
        self.fc2 = nn.Conv2d(s, c, 1)

    def forward(self, x):
        s = x.mean((2, 3), keepdim=True)
        return x * nn.functional.hardsigmoid(self.fc2(torch.relu(self.fc1(s))))


class Block(nn.Module):
    def __init__(self, cin, k, exp, cout, se, act, stride):
        super().__init__()
        a = nn.ReLU if act == "RE" else nn.Hardswish
        mods = []
        if exp != cin:
            mods.append(_cna(cin, exp, 1, act=a))
        mods.append(_cna(exp, exp, k, stride, groups=exp, act=a))
        if se:
            mods.append(SE(exp, _div8(exp // 4)))
        mods.append(_cna(exp, cout, 1))
        self.block = nn.Sequential(*mods)
        self.res = stride == 1 and cin == cout

    def forward(self, x):
        y = self.block(x)
        return y + x if self.res else y


LARGE = [
    (16, 3, 16, 16, False, "RE", 1), (16, 3, 64, 24, False, "RE", 2), (24, 3, 72, 24, False, "RE", 1),
    (24, 5, 72, 40, True, "RE", 2), (40, 5, 120, 40, True, "RE", 1), (40, 5, 120, 40, True, "RE", 1),
    (40, 3, 240, 80, False, "HS", 2), (80, 3, 200, 80, False, "HS", 1), (80, 3, 184, 80, False, "HS", 1),
    (80, 3, 184, 80, False, "HS", 1), (80, 3, 480, 112, True, "HS", 1), (112, 3, 672, 112, True, "HS", 1),
    (112, 5, 672, 160, True, "HS", 2), (160, 5, 960, 160, True, "HS", 1), (160, 5, 960, 160, True, "HS", 1),
]


class MobileNetV3Large(nn.Module):
    def __init__(self):
        super().__init__()
        self.features = nn.Sequential(_cna(3, 16, 3, 2, act=nn.Hardswish),
                                      *[Block(*c) for c in LARGE],
                                      _cna(160, 960, 1, act=nn.Hardswish))
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Linear(960, 1280), nn.Hardswish(), nn.Dropout(0.2),
                                        nn.Linear(1280, 1000))


class Encoder(nn.Module):
    """Input plus every `features` output: 18 tensors (reference :178-182)."""

    def __init__(self):
        super().__init__()
        self.original_model = MobileNetV3Large()

    def forward(self, x):
        feats = [x]
        for m in self.original_model.features:
            feats.append(m(feats[-1]))
        return feats


class PTModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.Unet = nn.Sequential(Encoder(), Decoder())

    def forward(self, x):
        return self.Unet(x)
