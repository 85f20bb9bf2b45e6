"""CPU restatement of GuideDepth = DDRNet-23-slim + 3 guided-upsampling blocks.

TEST INFRASTRUCTURE ONLY (see oracle/__init__).  Follows
src/GuideDepth/model/GuideDepth.py:9-57, modules.py:5-100 and
DDRNet_23_slim.py:35-365.  state_dict keys equal the reference's (471
entries), so fixtures and checkpoints are interchangeable.  Convolutions and
BatchNorm are ATen CPU modules; the resizes, SE and skip fusion use the
restated ops of oracle.ops.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops


def _bn(c):
    return nn.BatchNorm2d(c, momentum=0.1)


def _conv(cin, cout, k, stride=1, bias=False):
    return nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=bias)


class BasicBlock(nn.Module):
    """DDRNet_23_slim.py:41-72."""
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None, no_relu=False):
        super().__init__()
        self.conv1, self.bn1 = _conv(cin, planes, 3, stride), _bn(planes)
        self.conv2, self.bn2 = _conv(planes, planes, 3), _bn(planes)
        self.relu = nn.ReLU()
        self.downsample, self.no_relu = downsample, no_relu

    def forward(self, x):
        y = self.bn2(self.conv2(torch.relu(self.bn1(self.conv1(x)))))
        y = y + (x if self.downsample is None else self.downsample(x))
        return y if self.no_relu else torch.relu(y)


class Bottleneck(nn.Module):
    """DDRNet_23_slim.py:74-113 (expansion 2, no_relu default True)."""
    expansion = 2

    def __init__(self, cin, planes, stride=1, downsample=None, no_relu=True):
        super().__init__()
        self.conv1, self.bn1 = _conv(cin, planes, 1), _bn(planes)
        self.conv2, self.bn2 = _conv(planes, planes, 3, stride), _bn(planes)
        self.conv3, self.bn3 = _conv(planes, planes * 2, 1), _bn(planes * 2)
        self.relu = nn.ReLU()
        self.downsample, self.no_relu = downsample, no_relu

    def forward(self, x):
        y = torch.relu(self.bn1(self.conv1(x)))
        y = torch.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        y = y + (x if self.downsample is None else self.downsample(x))
        return y if self.no_relu else torch.relu(y)


def _stage(block, cin, planes, blocks, stride=1):
    """DualResNet._make_layer (DDRNet_23_slim.py:291-309)."""
    ds = None
    if stride != 1 or cin != planes * block.expansion:
        ds = nn.Sequential(nn.Conv2d(cin, planes * block.expansion, 1, stride=stride, bias=False),
                           _bn(planes * block.expansion))
    mods = [block(cin, planes, stride, ds)]
    for i in range(1, blocks):
        mods.append(block(planes * block.expansion, planes, 1, no_relu=(i == blocks - 1)))
    return nn.Sequential(*mods)


def _bn_relu_conv(cin, cout, k, pool=None):
    mods = ([pool] if pool is not None else []) + [_bn(cin), nn.ReLU(), _conv(cin, cout, k)]
    return nn.Sequential(*mods)


class DAPPM(nn.Module):
    """DDRNet_23_slim.py:115-195."""

    def __init__(self, cin, branch, cout):
        super().__init__()
        self.scale1 = _bn_relu_conv(cin, branch, 1, nn.AvgPool2d(5, 2, 2))
        self.scale2 = _bn_relu_conv(cin, branch, 1, nn.AvgPool2d(9, 4, 4))
        self.scale3 = _bn_relu_conv(cin, branch, 1, nn.AvgPool2d(17, 8, 8))
        self.scale4 = _bn_relu_conv(cin, branch, 1, nn.AdaptiveAvgPool2d((1, 1)))
        self.scale0 = _bn_relu_conv(cin, branch, 1)
        for i in range(1, 5):
            setattr(self, f"process{i}", _bn_relu_conv(branch, branch, 3))
        self.compression = _bn_relu_conv(branch * 5, cout, 1)
        self.shortcut = _bn_relu_conv(cin, cout, 1)

    def forward(self, x):
        h, w = x.shape[-2:]
        outs = [self.scale0(x)]
        for i in range(1, 5):
            up = ops.bilinear(getattr(self, f"scale{i}")(x), size=(h, w))
            outs.append(getattr(self, f"process{i}")(up + outs[-1]))
        return self.compression(torch.cat(outs, 1)) + self.shortcut(x)


class SegmentHead(nn.Module):
    """segmenthead (DDRNet_23_slim.py:198-219), scale_factor None."""

    def __init__(self, cin, mid, cout):
        super().__init__()
        self.bn1, self.conv1 = _bn(cin), _conv(cin, mid, 3)
        self.bn2, self.conv2 = _bn(mid), nn.Conv2d(mid, cout, 1, bias=True)
        self.relu = nn.ReLU()

    def forward(self, x):
        return self.conv2(torch.relu(self.bn2(self.conv1(torch.relu(self.bn1(x))))))


class DualResNet(nn.Module):
    """DualResNet(BasicBlock, [2,2,2,2], planes=32, spp 128, head 64) — DDRNet_23_slim.py:221-365."""

    def __init__(self, features=64, planes=32, spp_planes=128, head_planes=64):
        super().__init__()
        hp = planes * 2
        self.conv1 = nn.Sequential(_conv(3, planes, 3, 2, bias=True), _bn(planes), nn.ReLU(),
                                   _conv(planes, planes, 3, 2, bias=True), _bn(planes), nn.ReLU())
        self.relu = nn.ReLU()
        self.layer1 = _stage(BasicBlock, planes, planes, 2)
        self.layer2 = _stage(BasicBlock, planes, planes * 2, 2, 2)
        self.layer3 = _stage(BasicBlock, planes * 2, planes * 4, 2, 2)
        self.layer4 = _stage(BasicBlock, planes * 4, planes * 8, 2, 2)
        self.compression3 = nn.Sequential(_conv(planes * 4, hp, 1), _bn(hp))
        self.compression4 = nn.Sequential(_conv(planes * 8, hp, 1), _bn(hp))
        self.down3 = nn.Sequential(_conv(hp, planes * 4, 3, 2), _bn(planes * 4))
        self.down4 = nn.Sequential(_conv(hp, planes * 4, 3, 2), _bn(planes * 4), nn.ReLU(),
                                   _conv(planes * 4, planes * 8, 3, 2), _bn(planes * 8))
        self.layer3_ = _stage(BasicBlock, planes * 2, hp, 2)
        self.layer4_ = _stage(BasicBlock, hp, hp, 2)
        self.layer5_ = _stage(Bottleneck, hp, hp, 1)
        self.layer5 = _stage(Bottleneck, planes * 8, planes * 8, 1, 2)
        self.spp = DAPPM(planes * 16, spp_planes, planes * 4)
        self.final_layer = SegmentHead(planes * 4, head_planes, features)

    def forward(self, x):
        size = (x.shape[-2] // 8, x.shape[-1] // 8)
        r = torch.relu
        x = self.layer1(self.conv1(x))
        l2 = self.layer2(r(x))
        l3 = self.layer3(r(l2))
        hi = self.layer3_(r(l2))
        lo = l3 + self.down3(r(hi))
        hi = hi + ops.bilinear(self.compression3(r(l3)), size=size)
        l4 = self.layer4(r(lo))
        hi = self.layer4_(r(hi))
        lo = l4 + self.down4(r(hi))
        hi = hi + ops.bilinear(self.compression4(r(l4)), size=size)
        hi = self.layer5_(r(hi))
        lo = ops.bilinear(self.spp(self.layer5(r(lo))), size=size)
        return self.final_layer(lo + hi)


def _cbr(cin, cout, k):
    return [nn.Conv2d(cin, cout, k, padding=k // 2), _bn(cout), nn.ReLU()]


class SELayer(nn.Module):
    """modules.py:5-25."""

    def __init__(self, channel, reduction=16):
        super().__init__()
        self.fc = nn.Sequential(nn.Linear(channel, channel // reduction, bias=False), nn.ReLU(),
                                nn.Linear(channel // reduction, channel, bias=False), nn.Sigmoid())

    def forward(self, x):
        return ops.se(x, self.fc[0].weight, self.fc[2].weight)


class GuidedUpsamplingBlock(nn.Module):
    """Guided_Upsampling_Block (modules.py:29-100)."""

    def __init__(self, in_features, expand_features, out_features, kernel_size=3,
                 channel_attention=True, guidance_type="full", guide_features=3):
        super().__init__()
        e, k = expand_features, kernel_size
        self.channel_attention, self.guidance_type = channel_attention, guidance_type
        self.feature_conv = nn.Sequential(*_cbr(in_features, e, k), *_cbr(e, e // 2, 1))
        if guidance_type == "full":
            self.guide_conv = nn.Sequential(*_cbr(guide_features, e, k), *_cbr(e, e // 2, 1))
            comb = (e // 2) * 2
        elif guidance_type == "raw":
            comb = e // 2 + guide_features
        else:
            comb = e // 2
        self.comb_conv = nn.Sequential(*_cbr(comb, e, k), *_cbr(e, in_features, 1))
        self.reduce = nn.Conv2d(in_features, out_features, 1)
        if channel_attention:
            self.SE_block = SELayer(comb, reduction=1)

    def forward(self, guide, depth):
        x = self.feature_conv(depth)
        if self.guidance_type == "full":
            x = torch.cat([x, self.guide_conv(guide)], 1)
        elif self.guidance_type == "raw":
            x = torch.cat([x, guide], 1)
        if self.channel_attention:
            x = self.SE_block(x)
        return ops.skip_reduce(self.comb_conv(x), depth, self.reduce.weight, self.reduce.bias)


class GuideDepth(nn.Module):
    """GuideDepth.py:9-57 (pretrained weights are never loaded by the oracle)."""

    def __init__(self, up_features=(64, 32, 16), inner_features=(64, 32, 16)):
        super().__init__()
        u, e = list(up_features), list(inner_features)
        self.feature_extractor = DualResNet(features=u[0])
        self.up_1 = GuidedUpsamplingBlock(u[0], e[0], u[1])
        self.up_2 = GuidedUpsamplingBlock(u[1], e[1], u[2])
        self.up_3 = GuidedUpsamplingBlock(u[2], e[2], 1)

    def forward(self, x):
        y = self.feature_extractor(x)
        half, quarter = ops.nearest(x, scale_factor=0.5), ops.nearest(x, scale_factor=0.25)
        y = self.up_1(quarter, ops.bilinear(y, scale_factor=2))
        y = self.up_2(half, ops.bilinear(y, scale_factor=2))
        return self.up_3(x, ops.bilinear(y, scale_factor=2))
