"""SAM cross-window attention blocks of src/SAM.py on MI355X.

Same module tree, constructor signatures and state_dict keys as the
reference (WindowAttention :62-144, SAMBLOCK :146-244, SAM :247-309).  The
difference from NewCRF's layers: queries come from one stream (x, the
decoder) and keys / values from the other (v, the encoder features), v IS
projected (the kv Linear), and there is no shifted window.  The block runs
token-major with no padded / partitioned copies: LayerNorm (HIP), the q and
kv Linears (hipBLASLt) on the real tokens, then the HIP/MFMA window-attention
kernel of newcrf_layers.py, which takes a zero-padded token's q / k / v as the
Linears' biases (the reference pads after the LayerNorms, before the
Linears, SAM.py:214-229) -- here v_bias is the kv Linear's v half.
"""
from __future__ import annotations

import torch
from torch import nn

from .newcrf_layers import (LayerNorm, Mlp, _relative_position_index, linear_tok, nchw_to_tokens,
                            tokens_to_nchw, to_2tuple, window_attention, window_partition,
                            window_reverse)

__all__ = ["Mlp", "window_partition", "window_reverse", "WindowAttention", "SAMBLOCK", "SAM"]


class WindowAttention(nn.Module):
    """Window attention with q from x and k, v from the other stream (reference :62-144)."""

    def __init__(self, dim, window_size, num_heads, v_dim, qkv_bias=True, qk_scale=None,
                 attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim = dim
        self.window_size = to_2tuple(window_size)
        self.num_heads = num_heads
        head_dim = dim // num_heads
        if qk_scale is not None and qk_scale != head_dim ** -0.5:
            raise NotImplementedError("the HIP kernel uses the reference's head_dim ** -0.5 scale")
        if not qkv_bias:
            raise NotImplementedError("qkv_bias=False has no HIP kernel (padded tokens use the bias)")
        if v_dim != dim:
            raise NotImplementedError("SAM builds its block with v_dim == dim (SAM.py:273)")
        self.scale = head_dim ** -0.5
        wh, ww = self.window_size
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * wh - 1) * (2 * ww - 1), num_heads))
        self.register_buffer("relative_position_index", _relative_position_index(wh, ww))
        self.kv = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.q = nn.Linear(dim, dim, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(v_dim, v_dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02, a=-2.0, b=2.0)
        self.softmax = nn.Softmax(dim=-1)

    def forward_tokens(self, x_norm, v_norm, h, w):
        """x_norm, v_norm: [B, H*W, C] LayerNorm'd tokens -> proj(attention) [B, H*W, C]."""
        c = self.dim
        q = linear_tok(self.q, x_norm)
        kv = linear_tok(self.kv, v_norm)
        qk = torch.cat([q, kv[..., :c]], dim=-1)
        qk_bias = torch.cat([self.q.bias, self.kv.bias[:c]])
        v = kv[..., c:].contiguous().view(x_norm.shape[0], h, w, c)
        o = window_attention(qk, qk_bias, v, self.relative_position_bias_table, h, w,
                             self.num_heads, self.window_size[0], 0, v_bias=self.kv.bias[c:])
        return self.proj_drop(linear_tok(self.proj, o))


class SAMBLOCK(nn.Module):  # noqa: N801  (reference class name)
    """LN(x), LN(v) -> window cross-attention (+ residual) -> LN -> MLP (+ residual) (:146-244)."""

    def __init__(self, dim, num_heads, v_dim, window_size=7, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=LayerNorm):
        super().__init__()
        if drop_path > 0.0:
            raise NotImplementedError("stochastic depth (drop_path > 0) is not on the training path")
        self.window_size = window_size
        self.dim = dim
        self.num_heads = num_heads
        self.v_dim = v_dim
        self.mlp_ratio = mlp_ratio
        self.norm1 = LayerNorm(dim)
        self.normv = LayerNorm(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(window_size), num_heads=num_heads,
                                    v_dim=v_dim, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                    attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = LayerNorm(v_dim)
        self.mlp = Mlp(in_features=v_dim, hidden_features=int(v_dim * mlp_ratio), act_layer=nn.GELU,
                       drop=drop)

    def forward(self, x, v, H, W):  # noqa: N803
        """x, v: [B, H*W, C] token-major -> ([B, H*W, C], H, W)."""
        b, l, c = x.shape
        assert l == H * W, "input feature has wrong size"
        x = x + self.attn.forward_tokens(self.norm1(x), self.normv(v), H, W)
        x = x + self.mlp(self.norm2(x))
        return x, H, W


class SAM(nn.Module):
    """Cross-attention decoder stage (reference :247-309)."""

    def __init__(self, input_dim=96, embed_dim=96, v_dim=64, window_size=7, num_heads=4,
                 patch_size=4, in_chans=3, norm_layer=LayerNorm, patch_norm=True):
        super().__init__()
        self.embed_dim = embed_dim
        self.proj_e = nn.Conv2d(input_dim, embed_dim, 3, padding=1) if input_dim != embed_dim else None
        if v_dim != embed_dim:
            self.proj_q = nn.Conv2d(v_dim, embed_dim, 3, padding=1)
        elif embed_dim % v_dim == 0:
            self.proj_q = None
        # defined but never used by the reference's forward (SAM.py:271); kept for the keys
        self.proj = nn.Conv2d(embed_dim, embed_dim, 3, padding=1)
        v_dim = embed_dim
        self.sam_block = SAMBLOCK(dim=embed_dim, num_heads=num_heads, v_dim=v_dim,
                                  window_size=window_size, mlp_ratio=4.0, qkv_bias=True,
                                  qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0,
                                  norm_layer=norm_layer)
        self.add_module("norm_sam", LayerNorm(embed_dim))

    def forward(self, e, q):
        if self.proj_q is not None:
            q = self.proj_q(q)
        if self.proj_e is not None:
            e = self.proj_e(e)
        e_proj, q_proj = e, q
        wh, ww = q.size(2), q.size(3)
        q_out, h, w = self.sam_block(nchw_to_tokens(q), nchw_to_tokens(e), wh, ww)
        q_out = tokens_to_nchw(self.norm_sam(q_out), h, w)
        return q_out + e_proj + q_proj
