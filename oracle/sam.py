"""CPU restatement of the SAM decoder (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Follows src/SAM.py:62-309 (WindowAttention with separate q / kv Linears,
SAMBLOCK, SAM) and the Decoder of src/model_mobileV3_large_SAM.py:60-158.
Both streams are LayerNorm'd, zero-padded to multiples of the window AFTER
the norms (so a padded token's q, k and v are the Linears' biases), windowed,
attended without shift or mask, reversed and cropped.  state_dict keys match
the reference (including SAM.proj, which its forward never uses).  Pinned to
tests/golden/golden_sam.npz (the reference's own modules run here).
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops
from .newcrf import Mlp, from_windows, relative_position_index, to_windows


class WindowAttention(nn.Module):
    """q = Linear(C, C)(x), (k, v) = Linear(C, 2C)(v) per head; S = q k^T / sqrt(d) +
    T[index]; O = softmax(S) v; proj = Linear(C, C) (SAM.py:111-144)."""

    def __init__(self, dim, ws, heads):
        super().__init__()
        self.dim, self.ws, self.heads = dim, ws, heads
        self.scale = (dim // heads) ** -0.5
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.kv = nn.Linear(dim, dim * 2)
        self.q = nn.Linear(dim, dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, xw, vw):
        bw, n, c = xw.shape
        h, d = self.heads, c // self.heads
        q = self.q(xw).view(bw, n, h, d).transpose(1, 2) * self.scale
        kv = self.kv(vw).view(bw, n, 2, h, d)
        k, v = kv[:, :, 0].transpose(1, 2), kv[:, :, 1].transpose(1, 2)
        s = q @ k.transpose(-2, -1)
        bias = self.relative_position_bias_table[self.relative_position_index.reshape(-1)]
        s = s + bias.view(n, n, h).permute(2, 0, 1).unsqueeze(0)
        o = torch.softmax(s, dim=-1) @ v
        return self.proj(o.transpose(1, 2).reshape(bw, n, c))


class SAMBLOCK(nn.Module):  # noqa: N801
    def __init__(self, dim, heads, ws=7, mlp_ratio=4.0):
        super().__init__()
        self.ws = ws
        self.norm1 = nn.LayerNorm(dim)
        self.normv = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, ws, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x, v, h, w):
        """x, v: [B, H*W, C] tokens (SAM.py:195-244)."""
        b, l, c = x.shape
        ws = self.ws
        pad_b, pad_r = (ws - h % ws) % ws, (ws - w % ws) % ws
        t = torch.nn.functional.pad(self.norm1(x).view(b, h, w, c), (0, 0, 0, pad_r, 0, pad_b))
        vv = torch.nn.functional.pad(self.normv(v).view(b, h, w, c), (0, 0, 0, pad_r, 0, pad_b))
        hp, wp = h + pad_b, w + pad_r
        o = from_windows(self.attn(to_windows(t, ws), to_windows(vv, ws)), ws, hp, wp)
        x = x + o[:, :h, :w].reshape(b, h * w, c)
        return x + self.mlp(self.norm2(x))


class SAM(nn.Module):
    """SAM.py:247-309: out = norm(block(q, e)) + e_proj + q_proj."""

    def __init__(self, input_dim=96, embed_dim=96, v_dim=64, window_size=7, num_heads=4):
        super().__init__()
        self.embed_dim = embed_dim
        self.proj_e = nn.Conv2d(input_dim, embed_dim, 3, padding=1) if input_dim != embed_dim else None
        self.proj_q = nn.Conv2d(v_dim, embed_dim, 3, padding=1) if v_dim != embed_dim else None
        self.proj = nn.Conv2d(embed_dim, embed_dim, 3, padding=1)
        self.sam_block = SAMBLOCK(embed_dim, num_heads, window_size)
        self.norm_sam = nn.LayerNorm(embed_dim)

    def forward(self, e, q):
        if self.proj_q is not None:
            q = self.proj_q(q)
        if self.proj_e is not None:
            e = self.proj_e(e)
        b, c, h, w = q.shape
        out = self.sam_block(q.flatten(2).transpose(1, 2), e.flatten(2).transpose(1, 2), h, w)
        out = self.norm_sam(out).view(b, h, w, c).permute(0, 3, 1, 2)
        return out + e + q


class Decoder(nn.Module):
    """model_mobileV3_large_SAM.py:60-158."""

    def __init__(self):
        super().__init__()
        heads, crf, vd, ind = [4, 8, 16, 32], [128, 256, 512, 1024], [64, 128, 256, 512], [24, 40, 112, 160, 960]
        self.conv0 = nn.Conv2d(ind[4], vd[3], 1)
        for i in (3, 2, 1, 0):
            setattr(self, f"crf{i}", SAM(input_dim=ind[i], embed_dim=crf[i], window_size=7,
                                         v_dim=vd[i], num_heads=heads[i]))
        self.conv1 = nn.Conv2d(crf[0], 1, 3, padding=1)
        self.sigmoid = nn.Sigmoid()

    def forward(self, feats):
        e = self.crf3(feats[16], self.conv0(feats[17]))
        e = self.crf2(feats[13], torch.nn.functional.pixel_shuffle(e, 2))
        e = self.crf1(feats[7], torch.nn.functional.pixel_shuffle(e, 2))
        e = self.crf0(feats[4], torch.nn.functional.pixel_shuffle(e, 2))
        return ops.bilinear(self.sigmoid(self.conv1(e)), scale_factor=4)
