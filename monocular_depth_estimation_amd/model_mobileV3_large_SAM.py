"""MobileNetV3-Large + SAM depth model on MI355X (drop-in for src/model_mobileV3_large_SAM.py).

The model test.py evaluates (test.py:15,44).  Decoder (reference :60-158):
1x1 bridge 960->512, four SAM cross-attention stages (queries from the
decoder stream, keys / values from the encoder feature) with PixelShuffle(2)
between them, 3x3 conv -> sigmoid -> bilinear x4.  Encoder (:161-182): the
same MobileNetV3-Large feature list as the NewCRF model, but FROZEN -- the
reference sets requires_grad=False on every backbone parameter (:167-169),
so training updates the decoder only and the backward stops at the features.
"""
from __future__ import annotations

from torch import nn

from .model_mobileV3_large_newCRFs import Encoder as _NewCRFEncoder
from .model_mobileV3_large_newCRFs import upsample
from .SAM import SAM

__all__ = ["Decoder", "Encoder", "PTModel", "upsample"]


class Decoder(nn.Module):
    def __init__(self):
        super().__init__()
        num_heads = [4, 8, 16, 32]
        win = 7
        crf_dims = [128, 256, 512, 1024]
        v_dims = [64, 128, 256, 512]
        in_channels = [24, 40, 112, 160, 960]
        self.conv0 = nn.Conv2d(in_channels[4], v_dims[3], kernel_size=1, stride=1)
        for i in (3, 2, 1, 0):
            setattr(self, f"crf{i}", SAM(input_dim=in_channels[i], embed_dim=crf_dims[i],
                                         window_size=win, v_dim=v_dims[i], num_heads=num_heads[i]))
        self.conv1 = nn.Conv2d(crf_dims[0], 1, 3, padding=1)
        self.sigmoid = nn.Sigmoid()
        self.shuffle = nn.PixelShuffle(2)

    def forward(self, feats):
        """feats: the 18-entry list of Encoder.forward; uses feats[4, 7, 13, 16, 17]."""
        for i, c in ((4, 24), (7, 40), (13, 112), (16, 160), (17, 960)):
            if feats[i].shape[1] != c:
                raise ValueError(f"feats[{i}] has {feats[i].shape[1]} channels, expected {c}")
        e = self.crf3(feats[16], self.conv0(feats[17]))
        e = self.crf2(feats[13], self.shuffle(e))
        e = self.crf1(feats[7], self.shuffle(e))
        e = self.crf0(feats[4], self.shuffle(e))
        return upsample(self.sigmoid(self.conv1(e)), scale_factor=4)


class Encoder(_NewCRFEncoder):
    def __init__(self, pretrained=False):
        super().__init__(pretrained)
        for p in self.original_model.parameters():  # reference :167-169
            p.requires_grad_(False)


class PTModel(nn.Module):
    def __init__(self, pretrained=False):
        super().__init__()
        self.Unet = nn.Sequential(Encoder(pretrained), Decoder())

    def forward(self, x):
        return self.Unet(x)
