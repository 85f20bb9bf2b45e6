"""MobileNetV3-Large + NewCRF depth model on MI355X (drop-in for src/model_mobileV3_large_newCRFs.py).

Decoder (reference :60-158): 1x1 bridge 960->512, four NewCRF stages with
PixelShuffle(2) between them, 3x3 conv -> sigmoid -> bilinear x4.  The NewCRF
window attention runs on the HIP/MFMA kernel (newcrf_layers.py), the final
x4 upsample on the HIP resize kernel.

Encoder (reference :161-182): the reference wraps torchvision's
mobilenet_v3_large(pretrained=True) and returns the input plus the output of
every `features` module.  torchvision is not part of this stack (and the
pretrained fetch needs a network), so mobilenetv3.py restates the published
architecture with the same module tree and state_dict keys; its parity is
UNPINNED (no reference oracle can run here).  The unused classifier head is
kept for checkpoint compatibility but frozen (requires_grad=False) so
data-parallel training has no unused trainable parameters.
"""
from __future__ import annotations

import torch
from torch import nn

from .functional import bilinear_resize
from .mobilenetv3 import mobilenet_v3_large
from .nn import Conv2d
from .newcrf_layers import NewCRF


def upsample(x, scale_factor=2, mode="bilinear", align_corners=False):
    """F.interpolate(x, scale_factor, mode='bilinear') on the HIP kernel (reference :55-58)."""
    if mode != "bilinear":
        raise NotImplementedError(mode)
    return bilinear_resize(x, scale_factor=scale_factor, align_corners=align_corners)


class Decoder(nn.Module):
    def __init__(self):
        super().__init__()
        num_heads = [4, 8, 16, 32]
        win = 7
        crf_dims = [128, 256, 512, 1024]
        v_dims = [64, 128, 256, 512]
        in_channels = [24, 40, 112, 160, 960]
        # nn.py's Conv2d (same keys): the 1x1 bridge on the HIP 1x1 kernel + bias
        self.conv0 = Conv2d(in_channels[4], v_dims[3], kernel_size=1, stride=1)
        for i in (3, 2, 1, 0):
            setattr(self, f"crf{i}", NewCRF(input_dim=in_channels[i], embed_dim=crf_dims[i],
                                            window_size=win, v_dim=v_dims[i], num_heads=num_heads[i]))
        self.conv1 = Conv2d(crf_dims[0], 1, 3, padding=1)  # head.hip (nn.py Conv2d)
        self.sigmoid = nn.Sigmoid()
        self.shuffle = nn.PixelShuffle(2)

    def forward(self, feats):
        """feats: the 18-entry list of Encoder.forward; uses feats[4, 7, 13, 16, 17]."""
        for i, c in ((4, 24), (7, 40), (13, 112), (16, 160), (17, 960)):
            if feats[i].shape[1] != c:
                raise ValueError(f"feats[{i}] has {feats[i].shape[1]} channels, expected {c}")
        h, w = feats[4].shape[-2:]
        if (h * 4) % 32 or (w * 4) % 32:
            raise ValueError("the NewCRF decoder needs an input whose H and W are multiples of 32")
        e = self.crf3(feats[16], self.conv0(feats[17]))
        e = self.crf2(feats[13], self.shuffle(e))
        e = self.crf1(feats[7], self.shuffle(e))
        e = self.crf0(feats[4], self.shuffle(e))
        return upsample(self.sigmoid(self.conv1(e)), scale_factor=4)


class Encoder(nn.Module):
    def __init__(self, pretrained=False):
        super().__init__()
        if pretrained:
            raise NotImplementedError(
                "ImageNet MobileNetV3 weights are a network download in the reference "
                "(torchvision); load a state_dict instead")
        self.original_model = mobilenet_v3_large()
        for p in self.original_model.classifier.parameters():
            p.requires_grad_(False)

    def forward(self, x):
        features = [x]
        for _, v in self.original_model.features._modules.items():
            features.append(v(features[-1]))
        return features


class PTModel(nn.Module):
    def __init__(self, pretrained=False):
        super().__init__()
        self.Unet = nn.Sequential(Encoder(pretrained), Decoder())

    def forward(self, x):
        return self.Unet(x)
