"""CPU restatement of the NewCRF decoder (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Follows src/newcrf_layers.py:9-434 (Mlp, window partition/reverse,
WindowAttention, CRFBlock, BasicCRFLayer, NewCRF) and the Decoder of
src/model_mobileV3_large_newCRFs.py:60-158.  Written as explicit index
algebra on token-major tensors: padding to multiples of the window happens
after norm1 with zeros (so padded tokens still get q = k = qk bias and take
part in attention as keys), the cyclic shift is a torch.roll, and both CRF
blocks of a layer attend over the SAME v.  state_dict keys match the
reference.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import ops


def relative_position_index(ws: int) -> torch.Tensor:
    """(dy + ws - 1) * (2 ws - 1) + (dx + ws - 1) for every (query, key) pair."""
    ys, xs = np.meshgrid(np.arange(ws), np.arange(ws), indexing="ij")
    y, x = ys.reshape(-1), xs.reshape(-1)
    dy = y[:, None] - y[None, :] + ws - 1
    dx = x[:, None] - x[None, :] + ws - 1
    return torch.from_numpy((dy * (2 * ws - 1) + dx).astype(np.int64))


def shift_mask(hp: int, wp: int, ws: int, shift: int) -> torch.Tensor:
    """-100 between tokens of different shifted regions, [nW, ws*ws, ws*ws] (newcrf_layers.py:331-350)."""
    lab = np.zeros((hp, wp), dtype=np.float32)
    cuts = lambda n: [(0, n - ws), (n - ws, n - shift), (n - shift, n)]
    k = 0
    for a0, a1 in cuts(hp):
        for b0, b1 in cuts(wp):
            lab[a0:a1, b0:b1] = k
            k += 1
    win = lab.reshape(hp // ws, ws, wp // ws, ws).transpose(0, 2, 1, 3).reshape(-1, ws * ws)
    diff = win[:, None, :] - win[:, :, None]
    return torch.from_numpy(np.where(diff != 0, -100.0, 0.0).astype(np.float32))


def to_windows(t: torch.Tensor, ws: int) -> torch.Tensor:
    """[B, Hp, Wp, C] -> [B * nW, ws*ws, C] (window_partition, newcrf_layers.py:30-42)."""
    b, hp, wp, c = t.shape
    t = t.view(b, hp // ws, ws, wp // ws, ws, c).permute(0, 1, 3, 2, 4, 5)
    return t.reshape(-1, ws * ws, c)


def from_windows(t: torch.Tensor, ws: int, hp: int, wp: int) -> torch.Tensor:
    """Inverse of to_windows (window_reverse, newcrf_layers.py:45-59)."""
    b = t.shape[0] // ((hp // ws) * (wp // ws))
    t = t.view(b, hp // ws, wp // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5)
    return t.reshape(b, hp, wp, -1)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1, self.act, self.fc2 = nn.Linear(dim, hidden), nn.GELU(), nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class WindowAttention(nn.Module):
    """q, k = Linear(C, 2C)(x) per head; S = q k^T / sqrt(d) + T[index] (+ mask);
    O = softmax(S) v_heads; proj = Linear(C, C) (newcrf_layers.py:62-149)."""

    def __init__(self, dim, ws, heads):
        super().__init__()
        self.dim, self.ws, self.heads = dim, ws, heads
        self.scale = (dim // heads) ** -0.5
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.qk = nn.Linear(dim, dim * 2)
        self.proj = nn.Linear(dim, dim)

    def forward(self, xw, vw, mask=None):
        bw, n, c = xw.shape
        h, d = self.heads, c // self.heads
        qk = self.qk(xw).view(bw, n, 2, h, d)
        q = qk[:, :, 0].transpose(1, 2) * self.scale
        k = qk[:, :, 1].transpose(1, 2)
        s = q @ k.transpose(-2, -1)
        bias = self.relative_position_bias_table[self.relative_position_index.reshape(-1)]
        s = s + bias.view(n, n, h).permute(2, 0, 1).unsqueeze(0)
        if mask is not None:
            nw = mask.shape[0]
            s = (s.view(bw // nw, nw, h, n, n) + mask[None, :, None]).view(bw, h, n, n)
        p = torch.softmax(s, dim=-1)
        o = p @ vw.view(bw, n, h, d).transpose(1, 2)
        return self.proj(o.transpose(1, 2).reshape(bw, n, c))


class CRFBlock(nn.Module):
    def __init__(self, dim, heads, ws=7, shift=0, mlp_ratio=4.0):
        super().__init__()
        self.ws, self.shift = ws, shift
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, ws, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x, v, h, w, mask):
        """x: [B, H*W, C] tokens; v: [B, H, W, C]; newcrf_layers.py:195-257."""
        b, l, c = x.shape
        ws, sh = self.ws, self.shift
        pad_b, pad_r = (ws - h % ws) % ws, (ws - w % ws) % ws
        t = torch.nn.functional.pad(self.norm1(x).view(b, h, w, c), (0, 0, 0, pad_r, 0, pad_b))
        vv = torch.nn.functional.pad(v, (0, 0, 0, pad_r, 0, pad_b))
        hp, wp = h + pad_b, w + pad_r
        if sh:
            t = torch.roll(t, (-sh, -sh), (1, 2))
            vv = torch.roll(vv, (-sh, -sh), (1, 2))
        o = self.attn(to_windows(t, ws), to_windows(vv, ws), mask if sh else None)
        o = from_windows(o, ws, hp, wp)
        if sh:
            o = torch.roll(o, (sh, sh), (1, 2))
        x = x + o[:, :h, :w].reshape(b, h * w, c)
        return x + self.mlp(self.norm2(x))


class BasicCRFLayer(nn.Module):
    def __init__(self, dim, depth, heads, ws=7):
        super().__init__()
        self.ws = ws
        self.blocks = nn.ModuleList([CRFBlock(dim, heads, ws, 0 if i % 2 == 0 else ws // 2)
                                     for i in range(depth)])

    def forward(self, x, v, h, w):
        hp, wp = -(-h // self.ws) * self.ws, -(-w // self.ws) * self.ws
        mask = shift_mask(hp, wp, self.ws, self.ws // 2).to(x.device)
        for blk in self.blocks:
            x = blk(x, v, h, w, mask)
        return x


class NewCRF(nn.Module):
    """newcrf_layers.py:367-434 (depth 2, window 7, mlp ratio 4)."""

    def __init__(self, input_dim=96, embed_dim=96, v_dim=64, window_size=7, num_heads=4, depth=2):
        super().__init__()
        self.embed_dim = embed_dim
        self.proj_x = nn.Conv2d(input_dim, embed_dim, 3, padding=1) if input_dim != embed_dim else None
        self.proj_v = nn.Conv2d(v_dim, embed_dim, 3, padding=1) if v_dim != embed_dim else None
        self.crf_layer = BasicCRFLayer(embed_dim, depth, num_heads, window_size)
        self.norm_crf = nn.LayerNorm(embed_dim)

    def forward(self, x, v):
        if self.proj_x is not None:
            x = self.proj_x(x)
        if self.proj_v is not None:
            v = self.proj_v(v)
        b, c, h, w = x.shape
        tok = x.flatten(2).transpose(1, 2)
        out = self.norm_crf(self.crf_layer(tok, v.permute(0, 2, 3, 1), h, w))
        return out.view(b, h, w, c).permute(0, 3, 1, 2).contiguous()


class Decoder(nn.Module):
    """model_mobileV3_large_newCRFs.py:60-158: bridge -> crf3..crf0 with PixelShuffle(2) -> conv -> sigmoid -> x4."""

    def __init__(self):
        super().__init__()
        heads, crf, vd, ind = [4, 8, 16, 32], [128, 256, 512, 1024], [64, 128, 256, 512], [24, 40, 112, 160, 960]
        self.conv0 = nn.Conv2d(ind[4], vd[3], 1)
        for i in (3, 2, 1, 0):
            setattr(self, f"crf{i}", NewCRF(input_dim=ind[i], embed_dim=crf[i], window_size=7,
                                            v_dim=vd[i], num_heads=heads[i]))
        self.conv1 = nn.Conv2d(crf[0], 1, 3, padding=1)
        self.sigmoid = nn.Sigmoid()

    def forward(self, feats):
        e = self.crf3(feats[16], self.conv0(feats[17]))
        e = self.crf2(feats[13], torch.nn.functional.pixel_shuffle(e, 2))
        e = self.crf1(feats[7], torch.nn.functional.pixel_shuffle(e, 2))
        e = self.crf0(feats[4], torch.nn.functional.pixel_shuffle(e, 2))
        return ops.bilinear(self.sigmoid(self.conv1(e)), scale_factor=4)
