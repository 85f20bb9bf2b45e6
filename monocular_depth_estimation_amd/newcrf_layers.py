"""NewCRF layers on MI355X (drop-in for src/newcrf_layers.py).

Same classes, constructor signatures and state_dict keys as the reference
(Mlp, WindowAttention, CRFBlock, BasicCRFLayer, NewCRF, window_partition,
window_reverse).  The window-attention core of every CRFBlock — pad, cyclic
shift, partition, QK^T + relative-position bias + shift mask, softmax, AV,
reverse, unshift, crop — is ONE HIP kernel on MFMA
(functional.window_attention); tokens stay in [B, H*W, C] order throughout,
so the reference's pad / roll / permute / contiguous copies disappear.
The qk / proj / MLP Linears' forward and data-gradient GEMMs are hipBLASLt's;
their weight gradients (the long token reductions) run on mde_linear_wgrad
with the bias gradient from the same reads, fc1's bias gradient together
with the GELU backward in one pass (mde_gelu_bwd_colsum) -- fp32 training;
under autocast the plain modules run.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _abi
from .functional import _amp_bwd, _amp_fwd, _gpu, _ws
from .nn import Conv2d as _HipConv2d


def to_2tuple(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _colsum(g2):
    """Sum over the token rows of a contiguous [T, N] fp32 gradient (a Linear's bias gradient)."""
    t, n = g2.shape
    gb = torch.empty(n, dtype=torch.float32, device=g2.device)
    ws = _ws(_abi.query("mde_colsum_workspace", t, n), g2)
    _abi.call("mde_colsum", _abi.ptr(g2), _abi.ptr(gb), t, n, _abi.ptr(ws), 0, _abi.stream_of(g2))
    return gb


LIN_WGRAD = os.environ.get("MDE_LIN_WGRAD", "1") != "0"  # A/B: 0 = hipBLASLt's g.t() @ x


def _wgrad(g2, x2, bias: bool):
    """(g2.t() @ x2, g2.sum(0) or None) of contiguous [T, M] / [T, N] fp32
    token rows on mde_linear_wgrad (split-K MFMA, the bias gradient from the
    same reads), or None when the shape is not one it takes."""
    t, m = g2.shape
    n = x2.shape[1]
    if m * n > 16 * 128 * 128:
        # > 16 output tiles: the library GEMM (with the TunableOp table,
        # gemm_table.py) fills the chip without a split and wins from 32
        # tiles on (19200 x 1024 x 512: 164 vs 188 us; tools/lin_bench.py,
        # profiles/r06_lin_wgrad.txt)
        return None
    nbytes = _abi.query("mde_linear_wgrad_workspace", t, m, n) if LIN_WGRAD else 0
    if not nbytes:
        return None
    gw = torch.empty((m, n), dtype=torch.float32, device=g2.device)
    gb = torch.empty(m, dtype=torch.float32, device=g2.device) if bias else None
    ws = _ws(nbytes, g2)
    _abi.call("mde_linear_wgrad", _abi.ptr(g2), _abi.ptr(x2), _abi.ptr(gw),
              _abi.ptr(gb) if bias else None, t, m, n, _abi.ptr(ws), 0, _abi.stream_of(g2))
    return gw, gb


def _tok_ok(x, *widths) -> bool:
    """The fused token-major path: fp32 CUDA tensors, no autocast, widths % 4 == 0."""
    return (x.is_cuda and x.dtype == torch.float32 and not torch.is_autocast_enabled()
            and all(int(n) % 4 == 0 for n in widths)
            and bool(_abi.query("mde_colsum_workspace", max(1, x.numel() // x.shape[-1]),
                                max(int(n) for n in widths))))


class _LinearTok(torch.autograd.Function):
    """F.linear(x, W, b) over tokens (hipBLASLt) whose backward sums the bias
    gradient with mde_colsum (one fixed-order pass over g) instead of
    autograd's `grad.sum(0)`; the two GEMMs are the ones autograd runs."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).contiguous()
        gx = (g2 @ weight).view(x.shape) if ctx.needs_input_grad[0] else None
        x2 = x.reshape(-1, x.shape[-1])
        fused = _wgrad(g2, x2.contiguous(), ctx.needs_input_grad[2]) if ctx.needs_input_grad[1] else None
        if fused is not None:
            gw, gb = fused
        else:
            gw = g2.t() @ x2 if ctx.needs_input_grad[1] else None
            gb = _colsum(g2) if ctx.needs_input_grad[2] else None
        return gx, gw, gb


class _LinearGelu(torch.autograd.Function):
    """gelu(F.linear(x, W1, b1)) (Mlp fc1 + nn.GELU, reference :9-27): the
    backward's GELU derivative (erf form) and fc1's bias gradient come from ONE
    pass (mde_gelu_bwd_colsum: read dh and a, write da, column-sum da)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        a = F.linear(x, weight, bias)
        ctx.save_for_backward(x, weight, a)
        return F.gelu(a)

    @staticmethod
    def backward(ctx, dh):
        x, weight, a = ctx.saved_tensors
        dh2 = dh.reshape(-1, dh.shape[-1]).contiguous()
        a2 = a.reshape(-1, a.shape[-1])
        t, n = dh2.shape
        da = torch.empty_like(a2)
        gb = torch.empty(n, dtype=torch.float32, device=dh.device)
        ws = _ws(_abi.query("mde_colsum_workspace", t, n), dh2)
        _abi.call("mde_gelu_bwd_colsum", _abi.ptr(dh2), _abi.ptr(a2), _abi.ptr(da), _abi.ptr(gb),
                  t, n, _abi.ptr(ws), 0, _abi.stream_of(dh2))
        gx = (da @ weight).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            fused = _wgrad(da, x2.contiguous(), False)
            gw = fused[0] if fused is not None else da.t() @ x2
        return gx, gw, gb if ctx.needs_input_grad[2] else None


def linear_tok(lin: nn.Linear, x):
    """lin(x) on the fused-bias-gradient path when it applies (fp32, bias present)."""
    if lin.bias is not None and _tok_ok(x, lin.out_features):
        return _LinearTok.apply(x, lin.weight, lin.bias)
    return lin(x)


class Mlp(nn.Module):
    """fc1 -> act -> dropout -> fc2 -> dropout (reference :9-27; dropout 0 on the path)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                 drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        fused = (type(self.act) is nn.GELU and self.act.approximate == "none"
                 and (self.drop.p == 0.0 or not self.training) and self.fc1.bias is not None
                 and self.fc2.bias is not None
                 and _tok_ok(x, self.fc1.out_features, self.fc2.out_features))
        if fused:
            return linear_tok(self.fc2, _LinearGelu.apply(x, self.fc1.weight, self.fc1.bias))
        return self.drop(self.fc2(self.drop(self.act(self.fc1(x)))))


def window_partition(x, window_size):
    """(B, H, W, C) -> (num_windows*B, ws, ws, C) (reference :30-42)."""
    b, h, w, c = x.shape
    x = x.view(b, h // window_size, window_size, w // window_size, window_size, c)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, window_size, window_size, c)


def window_reverse(windows, window_size, H, W):  # noqa: N803
    """(num_windows*B, ws, ws, C) -> (B, H, W, C) (reference :45-59)."""
    b = int(windows.shape[0] / (H * W / window_size / window_size))
    x = windows.view(b, H // window_size, W // window_size, window_size, window_size, -1)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(b, H, W, -1)


def _relative_position_index(wh, ww):
    ys, xs = np.meshgrid(np.arange(wh), np.arange(ww), indexing="ij")
    y, x = ys.reshape(-1), xs.reshape(-1)
    idx = (y[:, None] - y[None, :] + wh - 1) * (2 * ww - 1) + (x[:, None] - x[None, :] + ww - 1)
    return torch.from_numpy(idx.astype(np.int64))


class _WindowAttn(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, qk, qk_bias, v, v_bias, table, h, w, heads, window, shift):
        qk = qk.contiguous()
        v = v.contiguous()
        b, _, c2 = qk.shape
        c = c2 // 2
        out = torch.empty((b, h * w, c), dtype=qk.dtype, device=qk.device)
        _abi.call("mde_window_attn_fwd", _abi.ptr(qk), _abi.ptr(qk_bias), _abi.ptr(v),
                  _abi.ptr(v_bias), _abi.ptr(table), _abi.ptr(out), b, h, w, c, heads, window, shift,
                  _abi.dtype_code(qk), _abi.stream_of(qk))
        ctx.save_for_backward(qk, qk_bias, v, v_bias, table)
        ctx.meta = (h, w, heads, window, shift)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, gout):
        qk, qk_bias, v, v_bias, table = ctx.saved_tensors
        h, w, heads, window, shift = ctx.meta
        gout = gout.contiguous()
        b, _, c2 = qk.shape
        c = c2 // 2
        gqk = torch.empty_like(qk)
        gv = torch.empty_like(v)
        gtable = torch.empty_like(table)
        gbias = torch.empty_like(qk_bias)
        gvb = torch.empty_like(v_bias) if v_bias is not None else None
        ws = _ws(_abi.query("mde_window_attn_workspace", b, h, w, c, heads, window), qk)
        _abi.call("mde_window_attn_bwd", _abi.ptr(gout), _abi.ptr(qk), _abi.ptr(qk_bias),
                  _abi.ptr(v), _abi.ptr(v_bias), _abi.ptr(table), _abi.ptr(gqk), _abi.ptr(gv),
                  _abi.ptr(gtable), _abi.ptr(gbias), _abi.ptr(gvb), b, h, w, c, heads, window, shift,
                  _abi.ptr(ws), _abi.dtype_code(gout), _abi.stream_of(gout))
        return gqk, gbias, gv, gvb, gtable, None, None, None, None, None


class _Transpose(torch.autograd.Function):
    """[B, M, N] -> [B, N, M] on the HIP LDS-tiled transpose (its own adjoint)."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, x):
        x = x.contiguous()
        b, m, n = x.shape
        y = torch.empty((b, n, m), dtype=x.dtype, device=x.device)
        _abi.call("mde_transpose", _abi.ptr(x), _abi.ptr(y), b, m, n, _abi.dtype_code(x),
                  _abi.stream_of(x))
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        return _Transpose.apply(gy)


def nchw_to_tokens(x):
    """[B, C, H, W] -> contiguous [B, H*W, C] (x.flatten(2).transpose(1, 2) materialised)."""
    _gpu(x)
    b, c, h, w = x.shape
    return _Transpose.apply(x.reshape(b, c, h * w))


def tokens_to_nchw(t, h, w):
    """[B, H*W, C] -> contiguous [B, C, H, W] (view(-1, H, W, C).permute(0, 3, 1, 2).contiguous())."""
    _gpu(t)
    b, l, c = t.shape
    return _Transpose.apply(t).view(b, c, h, w)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, x, weight, bias, eps):
        x = x.contiguous()
        c = x.shape[-1]
        rows = x.numel() // c
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        _abi.call("mde_layernorm_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(bias), _abi.ptr(y),
                  _abi.ptr(mean), _abi.ptr(rstd), rows, c, float(eps), _abi.dtype_code(x),
                  _abi.stream_of(x))
        ctx.save_for_backward(x, weight, mean, rstd)
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        x, weight, mean, rstd = ctx.saved_tensors
        gy = gy.contiguous()
        c = x.shape[-1]
        rows = x.numel() // c
        gx = torch.empty_like(x)
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        ws = _ws(_abi.query("mde_layernorm_workspace", rows, c), x)
        _abi.call("mde_layernorm_bwd", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(weight), _abi.ptr(mean),
                  _abi.ptr(rstd), _abi.ptr(gx), _abi.ptr(gw), _abi.ptr(gb), rows, c, _abi.ptr(ws),
                  _abi.dtype_code(gy), _abi.stream_of(gy))
        return gx, gw, gb, None


class _AddLayerNorm(torch.autograd.Function):
    """(s, LayerNorm(s)) with s = x + r in ONE HIP pass (mde_layernorm_add_fwd):
    CRFBlock's residual adds, each followed by a LayerNorm
    (newcrf_layers.py:229-257,434).  The backward adds the gradient that s's
    residual branch carries in the LayerNorm backward's epilogue
    (mde_layernorm_bwd_res) and hands the sum to both x and r -- no separate
    add pass forward, no accumulation pass backward."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, x, r, weight, bias, eps):
        x = x.contiguous()
        r = r.contiguous()
        c = x.shape[-1]
        rows = x.numel() // c
        s = torch.empty_like(x)
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        _abi.call("mde_layernorm_add_fwd", _abi.ptr(x), _abi.ptr(r), _abi.ptr(weight), _abi.ptr(bias),
                  _abi.ptr(s), _abi.ptr(y), _abi.ptr(mean), _abi.ptr(rstd), rows, c, float(eps),
                  _abi.dtype_code(x), _abi.stream_of(x))
        ctx.save_for_backward(s, weight, mean, rstd)
        return s, y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gs, gy):
        s, weight, mean, rstd = ctx.saved_tensors
        gy = gy.contiguous()
        c = s.shape[-1]
        rows = s.numel() // c
        gx = torch.empty_like(s)
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        ws = _ws(_abi.query("mde_layernorm_workspace", rows, c), s)
        _abi.call("mde_layernorm_bwd_res", _abi.ptr(gy), _abi.ptr(s), _abi.ptr(gs.contiguous()),
                  _abi.ptr(weight), _abi.ptr(mean), _abi.ptr(rstd), _abi.ptr(gx), _abi.ptr(gw),
                  _abi.ptr(gb), rows, c, _abi.ptr(ws), _abi.dtype_code(gy), _abi.stream_of(gy))
        return gx, gx, gw, gb, None


LN_ADD = os.environ.get("MDE_LN_ADD", "1") != "0"  # A/B: 0 = separate add + LayerNorm


def add_layer_norm(x, r, norm):
    """(x + r, norm(x + r)): one HIP pass (_AddLayerNorm) where it applies."""
    if (LN_ADD and isinstance(norm, LayerNorm) and x.is_cuda and x.dtype == torch.float32
            and r.dtype == torch.float32 and x.shape == r.shape and not torch.is_autocast_enabled()
            and norm.weight is not None and norm.bias is not None
            and len(norm.normalized_shape) == 1 and x.shape[-1] == norm.normalized_shape[0]
            and _abi.query("mde_layernorm_workspace", max(1, x.numel() // x.shape[-1]),
                           x.shape[-1])):
        return _AddLayerNorm.apply(x, r, norm.weight, norm.bias, norm.eps)
    s = x + r
    return s, norm(s)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm over the last axis on the HIP kernel (same parameters and keys)."""

    def forward(self, x):
        _gpu(x)
        if (len(self.normalized_shape) != 1 or self.weight is None or self.bias is None
                or x.shape[-1] != self.normalized_shape[0]):
            raise NotImplementedError("the HIP LayerNorm covers affine LayerNorm(C) over the last axis")
        return _LayerNorm.apply(x, self.weight, self.bias, self.eps)


def window_attention(qk, qk_bias, v, table, h, w, heads, window, shift, v_bias=None):
    """Shifted-window attention core of CRFBlock on the HIP/MFMA kernel.

    qk: [B, H*W, 2C] (qk Linear of the real tokens), qk_bias: [2C], v: [B, H, W, C],
    table: [(2ws-1)^2, heads].  v_bias: [C] value of a padded token (SAM's
    projected v), None = 0 (NewCRF).  Returns [B, H*W, C] (before proj).
    """
    _gpu(qk, qk_bias, v, table)
    return _WindowAttn.apply(qk, qk_bias, v, v_bias, table, int(h), int(w), int(heads), int(window),
                             int(shift))


class WindowAttention(nn.Module):
    """Relative-position-biased window attention with an un-projected v (reference :62-149)."""

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
        self.scale = head_dim ** -0.5
        wh, ww = self.window_size
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * wh - 1) * (2 * ww - 1), num_heads))
        self.register_buffer("relative_position_index", _relative_position_index(wh, ww))
        self.qk = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(v_dim, v_dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02, a=-2.0, b=2.0)
        self.softmax = nn.Softmax(dim=-1)

    def forward_tokens(self, x_norm, v, h, w, shift):
        """x_norm: [B, H*W, C] LayerNorm'd tokens, v: [B, H, W, C] -> proj(attention) [B, H*W, C]."""
        qk = linear_tok(self.qk, x_norm)
        o = window_attention(qk, self.qk.bias, v, self.relative_position_bias_table, h, w,
                             self.num_heads, self.window_size[0], shift)
        return self.proj_drop(linear_tok(self.proj, o))


class CRFBlock(nn.Module):
    """LN -> shifted-window attention (+ residual) -> LN -> MLP (+ residual) (reference :152-257)."""

    def __init__(self, dim, num_heads, v_dim, window_size=7, shift_size=0, mlp_ratio=4.0,
                 qkv_bias=True, qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0,
                 act_layer=nn.GELU, norm_layer=LayerNorm):
        super().__init__()
        self.dim, self.num_heads, self.v_dim = dim, num_heads, v_dim
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        if drop_path > 0.0:
            raise NotImplementedError("stochastic depth (drop_path > 0) is not on the training path")
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(window_size), num_heads=num_heads,
                                    v_dim=v_dim, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                    attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(v_dim)
        self.mlp = Mlp(in_features=v_dim, hidden_features=int(v_dim * mlp_ratio), act_layer=act_layer,
                       drop=drop)
        self.H = None
        self.W = None

    def forward(self, x, v, mask_matrix=None):
        """x: [B, H*W, C]; v: [B, H, W, C]; the shift mask is computed in-kernel."""
        x1, m = self.forward_pending(x, None, v)
        return x1 + m

    def forward_pending(self, x, pending, v):
        """This block on x + pending (the previous block's MLP branch, not yet
        added): returns (x1, m) with the block's output x1 + m left un-added,
        so that the next LayerNorm adds it in its own pass (add_layer_norm).
        Same arithmetic as forward (reference :229-257)."""
        b, l, c = x.shape
        h, w = self.H, self.W
        assert l == h * w, "input feature has wrong size"
        if pending is None:
            n1 = self.norm1(x)
        else:
            x, n1 = add_layer_norm(x, pending, self.norm1)
        a = self.attn.forward_tokens(n1, v, h, w, self.shift_size)
        x1, n2 = add_layer_norm(x, a, self.norm2)
        return x1, self.mlp(n2)


class BasicCRFLayer(nn.Module):
    """`depth` CRFBlocks alternating W-MSA / SW-MSA over the same v (reference :260-363)."""

    def __init__(self, dim, depth, num_heads, v_dim, window_size=7, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=LayerNorm,
                 downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            CRFBlock(dim=dim, num_heads=num_heads, v_dim=v_dim, window_size=window_size,
                     shift_size=0 if (i % 2 == 0) else window_size // 2, mlp_ratio=mlp_ratio,
                     qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                     drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                     norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def _run(self, x, v, H, W):  # noqa: N803
        pending = None
        for blk in self.blocks:
            blk.H, blk.W = H, W
            x, pending = blk.forward_pending(x, pending, v)
        return x, pending

    def forward_norm(self, x, v, H, W, norm):  # noqa: N803
        """norm(self(x, v, H, W)[0]) with the last residual add inside the norm's pass."""
        x, pending = self._run(x, v, H, W)
        return norm(x) if pending is None else add_layer_norm(x, pending, norm)[1]

    def forward(self, x, v, H, W):  # noqa: N803
        x, pending = self._run(x, v, H, W)
        if pending is not None:
            x = x + pending
        if self.downsample is not None:
            return x, H, W, self.downsample(x, H, W), (H + 1) // 2, (W + 1) // 2
        return x, H, W, x, H, W


class NewCRF(nn.Module):
    """Neural window FC-CRF stage (reference :367-434)."""

    def __init__(self, input_dim=96, embed_dim=96, v_dim=64, window_size=7, num_heads=4, depth=2,
                 patch_size=4, in_chans=3, norm_layer=LayerNorm, patch_norm=True):
        super().__init__()
        self.embed_dim = embed_dim
        self.patch_norm = patch_norm
        # the projections on the HIP 3x3 kernels (Winograd forward / data
        # gradient where the channel counts allow, + bias), same state_dict keys
        self.proj_x = _HipConv2d(input_dim, embed_dim, 3, padding=1) if input_dim != embed_dim else None
        if v_dim != embed_dim:
            self.proj_v = _HipConv2d(v_dim, embed_dim, 3, padding=1)
        elif embed_dim % v_dim == 0:
            self.proj_v = None
        v_dim = embed_dim
        self.crf_layer = BasicCRFLayer(dim=embed_dim, depth=depth, num_heads=num_heads, v_dim=v_dim,
                                       window_size=window_size, mlp_ratio=4.0, qkv_bias=True,
                                       qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0,
                                       norm_layer=norm_layer, downsample=None, use_checkpoint=False)
        self.add_module("norm_crf", norm_layer(embed_dim))

    def forward(self, x, v):
        if self.proj_x is not None:
            x = self.proj_x(x)
        if self.proj_v is not None:
            v = self.proj_v(v)
        b, c, h, w = x.shape
        tokens = nchw_to_tokens(x)
        v_nhwc = nchw_to_tokens(v).view(b, h, w, -1)
        # crf_layer then norm_crf (reference :430-434), the last residual add
        # inside norm_crf's pass
        return tokens_to_nchw(self.crf_layer.forward_norm(tokens, v_nhwc, h, w, self.norm_crf), h, w)
