"""DDRNet-23-slim encoder of GuideDepth on MI355X.

Drop-in for src/GuideDepth/model/DDRNet_23_slim.py (DualResNet_Backbone,
:357-365): same constructor, same state_dict keys (333 `feature_extractor.*`
entries inside GuideDepth).  Dense 3x3/1x1 convolutions, BatchNorm and
average pools run on PyTorch-ROCm (MIOpen — MFMA-bound, not hand-kernel
targets); the seven bilinear resizes (:182-191 in DAPPM, :332, :342, :348)
run on the HIP resize kernel.

The reference's `depthwise` / `pointwise` helpers (:19-33) and `Interpolate`
(:367-375) are dead code there and are not reproduced.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from ...functional import bilinear_resize
from ...nn import BatchNorm2d, Conv2d, conv_nobias_stats, residual_grad_slot, run_sequential

BN_MOMENTUM = 0.1


def _bn(c, act="none"):
    """BatchNorm on the HIP kernel; act='relu' fuses the ReLU that follows it."""
    return BatchNorm2d(c, momentum=BN_MOMENTUM, act=act)


def conv3x3(in_planes, out_planes, stride=1):
    """3x3 convolution, padding 1, no bias (reference :35-38)."""
    return Conv2d(in_planes, out_planes, 3, stride=stride, padding=1, bias=False)


def _conv_stats(conv, x, bn, gx_slot=None):
    """(y, stats) positional arguments of bn: conv(x) without a bias and its BN
    statistics from the conv's epilogue (nn.conv_nobias_stats)."""
    y, st = conv_nobias_stats(conv, x, bn, gx_slot)
    return y, None, None, st


class BasicBlock(nn.Module):
    """Two 3x3 conv+BN, residual, optional final ReLU (reference :41-72).

    bn1 carries the ReLU; bn2 takes the residual and the final ReLU in the
    same pass (`out += residual; relu(out)` fused into the BN apply).
    """
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, no_relu=False):
        super().__init__()
        self.conv1, self.bn1 = conv3x3(inplanes, planes, stride), _bn(planes, "relu")
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _bn(planes, "none" if no_relu else "relu")
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.no_relu = no_relu
        # the final activation when the owner applies its own ReLU to this
        # block's output and reads nothing else of it (DualResNet: layer1 /
        # layer2); None = bn2's ("none" with no_relu, else "relu")
        self.out_act = None

    def forward(self, x):
        # bias-free 3x3 convs on the HIP kernels where they apply (conv_nobias);
        # in training each BN takes its batch statistics from the conv's epilogue
        # x feeds conv1 and (no downsample) the residual add: the residual's
        # gradient then reaches conv1's Winograd data gradient through a slot
        # and is summed in its epilogue instead of by an autograd add
        slot = residual_grad_slot(self.conv1, x) if self.downsample is None else None
        y = self.bn1(*_conv_stats(self.conv1, x, self.bn1, slot))
        res = x if self.downsample is None else run_sequential(self.downsample, x)
        y, st = conv_nobias_stats(self.conv2, y, self.bn2)
        return self.bn2(y, residual=res, stats=st, act=self.out_act, res_slot=slot)


class Bottleneck(nn.Module):
    """1x1 -> 3x3(stride) -> 1x1 (x2 channels), residual (reference :74-113)."""
    expansion = 2

    def __init__(self, inplanes, planes, stride=1, downsample=None, no_relu=True):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _bn(planes, "relu")
        self.conv2, self.bn2 = conv3x3(planes, planes, stride), _bn(planes, "relu")
        self.conv3 = Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = _bn(planes * self.expansion, "none" if no_relu else "relu")
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.no_relu = no_relu

    def forward(self, x):
        y = self.bn1(*_conv_stats(self.conv1, x, self.bn1))
        y = self.bn2(*_conv_stats(self.conv2, y, self.bn2))
        res = x if self.downsample is None else run_sequential(self.downsample, x)
        y, st = conv_nobias_stats(self.conv3, y, self.bn3)
        return self.bn3(y, residual=res, stats=st)


def _pre_act(cin, cout, k, pool=None):
    """[pool] -> BN+ReLU (fused; Identity keeps the ReLU slot) -> conv(k, bias=False)."""
    mods = [] if pool is None else [pool]
    mods += [_bn(cin, "relu"), nn.Identity(),
             Conv2d(cin, cout, k, padding=k // 2, bias=False)]
    return nn.Sequential(*mods)


class DAPPM(nn.Module):
    """Deep aggregation pyramid pooling (reference :115-195).

    Each pooled branch is bilinearly resized back to the input size on the HIP
    kernel (ratios such as 4x5 -> 8x10, 1x2 -> 8x10) before its 3x3 process.
    """

    _POOLS = {1: (5, 2, 2), 2: (9, 4, 4), 3: (17, 8, 8)}

    def __init__(self, inplanes, branch_planes, outplanes):
        super().__init__()
        for i, (k, s, p) in self._POOLS.items():
            setattr(self, f"scale{i}", _pre_act(inplanes, branch_planes, 1, nn.AvgPool2d(k, s, p)))
        self.scale4 = _pre_act(inplanes, branch_planes, 1, nn.AdaptiveAvgPool2d((1, 1)))
        self.scale0 = _pre_act(inplanes, branch_planes, 1)
        for i in range(1, 5):
            setattr(self, f"process{i}", _pre_act(branch_planes, branch_planes, 3))
        self.compression = _pre_act(branch_planes * 5, outplanes, 1)
        self.shortcut = _pre_act(inplanes, outplanes, 1)

    def forward(self, x):
        size = (x.shape[-2], x.shape[-1])
        branches = [self.scale0(x)]
        for i in range(1, 5):
            pooled = getattr(self, f"scale{i}")(x)
            branches.append(getattr(self, f"process{i}")(
                bilinear_resize(pooled, size=size) + branches[-1]))
        return self.compression(torch.cat(branches, 1)) + self.shortcut(x)


class segmenthead(nn.Module):  # noqa: N801  (reference class name)
    """BN-ReLU-3x3 -> BN-ReLU-1x1(bias) head (reference :198-219)."""

    def __init__(self, inplanes, interplanes, outplanes, scale_factor=None):
        super().__init__()
        self.bn1 = _bn(inplanes, "relu")
        self.conv1 = Conv2d(inplanes, interplanes, 3, padding=1, bias=False)
        self.bn2 = _bn(interplanes, "relu")
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = Conv2d(interplanes, outplanes, 1, padding=0, bias=True)
        self.scale_factor = scale_factor

    def forward(self, x):
        x = self.conv1(self.bn1(x))
        out = self.conv2(self.bn2(x))
        if self.scale_factor is not None:
            out = bilinear_resize(out, size=(x.shape[-2] * self.scale_factor,
                                             x.shape[-1] * self.scale_factor))
        return out


def _make_layer(block, inplanes, planes, blocks, stride=1):
    """Stage of `blocks` blocks; the last one has no final ReLU (reference :291-309)."""
    downsample = None
    if stride != 1 or inplanes != planes * block.expansion:
        downsample = nn.Sequential(
            Conv2d(inplanes, planes * block.expansion, 1, stride=stride, bias=False),
            _bn(planes * block.expansion))
    layers = [block(inplanes, planes, stride, downsample)]
    for i in range(1, blocks):
        layers.append(block(planes * block.expansion, planes, stride=1,
                            no_relu=(i == blocks - 1)))
    return nn.Sequential(*layers)


def _seq_bn_residual(seq, x, residual, act=None):
    """act(residual + seq(x)) for a Sequential ending in a BatchNorm: the add (and
    the activation, e.g. the ReLU the reference applies to the sum next) run in
    the BN pass.  Its bias-free convs go through conv_nobias (HIP kernels where
    they apply)."""
    mods = list(seq)
    conv = mods[-2] if len(mods) >= 2 else None
    if not (isinstance(conv, nn.Conv2d) and conv.bias is None):
        # conv_nobias_stats assumes a bias-free conv feeding the BN: anything else
        # (a biased conv, a non-conv module) runs as-is, the add still in the BN
        return mods[-1](run_sequential(mods[:-1], x), residual=residual, act=act)
    x = run_sequential(mods[:-2], x) if len(mods) > 2 else x
    y, st = conv_nobias_stats(conv, x, mods[-1])
    return mods[-1](y, residual=residual, stats=st, act=act)


class DualResNet(nn.Module):
    """Two-branch (low/high resolution) encoder with bilateral fusion (reference :221-354)."""

    def __init__(self, block, layers, out_features=19, planes=64, spp_planes=128,
                 head_planes=128, augment=False, skip_out=False):
        super().__init__()
        hp = planes * 2
        self.augment = augment
        self.skip_out = skip_out
        self.conv1 = nn.Sequential(
            nn.Conv2d(3, planes, 3, stride=2, padding=1), _bn(planes, "relu"), nn.Identity(),
            nn.Conv2d(planes, planes, 3, stride=2, padding=1), _bn(planes, "relu"), nn.Identity())
        self.relu = nn.ReLU(inplace=False)
        widths = [planes, planes, planes * 2, planes * 4, planes * 8]
        for i in range(4):
            setattr(self, f"layer{i + 1}",
                    _make_layer(block, widths[i], widths[i + 1], layers[i], stride=1 if i == 0 else 2))
        self.compression3 = nn.Sequential(Conv2d(planes * 4, hp, 1, bias=False), _bn(hp))
        self.compression4 = nn.Sequential(Conv2d(planes * 8, hp, 1, bias=False), _bn(hp))
        self.down3 = nn.Sequential(conv3x3(hp, planes * 4, 2), _bn(planes * 4))
        self.down4 = nn.Sequential(conv3x3(hp, planes * 4, 2), _bn(planes * 4, "relu"), nn.Identity(),
                                   conv3x3(planes * 4, planes * 8, 2), _bn(planes * 8))
        self.layer3_ = _make_layer(block, planes * 2, hp, 2)
        self.layer4_ = _make_layer(block, hp, hp, 2)
        self.layer5_ = _make_layer(Bottleneck, hp, hp, 1)
        self.layer5 = _make_layer(Bottleneck, planes * 8, planes * 8, 1, stride=2)
        self.spp = DAPPM(planes * 16, spp_planes, planes * 4)
        self.final_layer = segmenthead(planes * 4, head_planes, out_features)
        # layers[0] and layers[1] are only ever read through self.relu
        # (reference :319-327): their last BatchNorm applies that ReLU in its
        # own pass (no separate relu / threshold_backward launches)
        self.layer1[-1].out_act = "relu"
        self.layer2[-1].out_act = "relu"
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes the HIP BatchNorm2d
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        out_size = (x.shape[-2] // 8, x.shape[-1] // 8)
        r = self.relu
        # `relu(layers[0])` / `relu(layers[1])` come out of layer1 / layer2's last
        # BN (out_act); the reference takes relu(layers[1]) twice (:327, :329;
        # inplace=False): one tensor here
        rlow = self.layer1(run_sequential(self.conv1, x))  # conv biases folded into the BNs
        rl2 = self.layer2(rlow)
        l3 = self.layer3(rl2)
        high = self.layer3_(rl2)
        # relu(l3 + down3(relu(high))): the add and the ReLU of :336 in the BN pass
        rlow = _seq_bn_residual(self.down3, r(high), l3, act="relu")
        high = high + bilinear_resize(run_sequential(self.compression3, r(l3)), size=out_size)
        l4 = self.layer4(rlow)
        high = self.layer4_(r(high))
        rlow = _seq_bn_residual(self.down4, r(high), l4, act="relu")  # :344 / :350
        high = high + bilinear_resize(run_sequential(self.compression4, r(l4)), size=out_size)
        high = self.layer5_(r(high))
        low = bilinear_resize(self.spp(self.layer5(rlow)), size=out_size)
        return self.final_layer(low + high)


DEFAULT_WEIGHTS = os.path.join(".", "GuideDepth", "model", "weights", "DDRNet23s_imagenet.pth")


def DualResNet_Backbone(pretrained=False, features=64, weights_path=None):  # noqa: N802
    """DDRNet-23-slim as GuideDepth's encoder (reference :357-365).

    With pretrained=True the ImageNet blob is loaded non-strictly from
    `weights_path` (default: the reference's relative path, overridable with
    MDE_DDRNET_WEIGHTS) using torch.load(weights_only=True); a missing blob
    raises FileNotFoundError as the reference does.
    """
    model = DualResNet(BasicBlock, [2, 2, 2, 2], out_features=features, planes=32,
                       spp_planes=128, head_planes=64, augment=False)
    if pretrained:
        path = weights_path or os.environ.get("MDE_DDRNET_WEIGHTS", DEFAULT_WEIGHTS)
        state = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(state, strict=False)
    return model
