"""BatchNorm2d on the HIP kernels, with the following ReLU / residual add fused.

`BatchNorm2d(c, act="relu")` is an nn.BatchNorm2d (same parameters, buffers
and state_dict keys) whose forward runs mde_batchnorm_fwd_{train,eval} and
applies the activation — and optionally adds a residual first — in the same
streaming pass.  Where the reference writes `BN -> ReLU(inplace)` the ReLU
module slot is kept as an nn.Identity so Sequential indices (and therefore
state_dict keys) are unchanged.
"""
from __future__ import annotations

import contextlib
import os

import torch
from torch import nn

from . import _abi
from .functional import GradSlot, _amp_bwd, _amp_fwd, _gpu, _ws

_ACTS = {"none": 0, "relu": 1, "hardswish": 2}


# BN keeps a bf16 activation in bf16 (autocast convolutions produce and consume
# bf16; statistics and coefficients stay fp32 in the kernels), anything else in fp32.
_bn_fwd = torch.amp.custom_fwd(device_type="cuda")


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    @_bn_fwd
    def forward(ctx, x, weight, bias, prebias, residual, running_mean, running_var, nbt,
                training, momentum, eps, act, stats=None, res_slot=None):
        dt = torch.bfloat16 if x.dtype == torch.bfloat16 else torch.float32
        x = x.to(dt).contiguous()
        residual = residual.to(dt).contiguous() if residual is not None else None
        n, c, h, w = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(c, dtype=torch.float32, device=x.device)
        invstd = torch.empty(c, dtype=torch.float32, device=x.device)
        st = _abi.stream_of(x)
        if training and stats is not None:
            # statistics from the producing conv's epilogue: no stats pass over x
            ws = _ws(_abi.query("mde_batchnorm_workspace", n, c, h, w), x)
            _abi.call("mde_batchnorm_fwd_train_stats", _abi.ptr(x), _abi.ptr(weight),
                      _abi.ptr(bias), _abi.ptr(prebias), _abi.ptr(running_mean),
                      _abi.ptr(running_var), _abi.ptr(nbt), float(momentum), float(eps),
                      _abi.ptr(residual), _abi.ptr(y), _abi.ptr(mean), _abi.ptr(invstd), n, c, h,
                      w, act, _abi.ptr(stats), stats.shape[1], _abi.ptr(ws), _abi.dtype_code(x), st)
        elif training:
            ws = _ws(_abi.query("mde_batchnorm_workspace", n, c, h, w), x)
            _abi.call("mde_batchnorm_fwd_train", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(bias),
                      _abi.ptr(prebias), _abi.ptr(running_mean), _abi.ptr(running_var),
                      _abi.ptr(nbt), float(momentum), float(eps), _abi.ptr(residual), _abi.ptr(y),
                      _abi.ptr(mean), _abi.ptr(invstd), n, c, h, w, act, _abi.ptr(ws),
                      _abi.dtype_code(x), st)
        else:
            _abi.call("mde_batchnorm_fwd_eval", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(bias),
                      _abi.ptr(prebias), _abi.ptr(running_mean), _abi.ptr(running_var),
                      float(eps), _abi.ptr(residual), _abi.ptr(y), _abi.ptr(mean),
                      _abi.ptr(invstd), n, c, h, w, act, _abi.dtype_code(x), st)
        ctx.save_for_backward(x, weight, bias, residual, mean, invstd)
        ctx.training, ctx.act, ctx.has_prebias = bool(training), act, prebias is not None
        ctx.res_slot = res_slot
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        x, weight, bias, residual, mean, invstd = ctx.saved_tensors
        gy = gy.to(x.dtype).contiguous()
        n, c, h, w = x.shape
        gx = torch.empty_like(x)
        gw = torch.empty_like(weight) if ctx.needs_input_grad[1] else None
        gb = torch.empty_like(bias) if ctx.needs_input_grad[2] else None
        gpb = torch.empty_like(weight) if (ctx.has_prebias and ctx.needs_input_grad[3]) else None
        want_r = residual is not None and ctx.needs_input_grad[4]
        # with no activation the residual's gradient is gy itself: no write needed
        gr = torch.empty_like(x) if (want_r and ctx.act) else None
        ws = _ws(_abi.query("mde_batchnorm_workspace", n, c, h, w), x)
        _abi.call("mde_batchnorm_bwd", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(residual),
                  _abi.ptr(weight), _abi.ptr(bias), _abi.ptr(mean), _abi.ptr(invstd),
                  int(ctx.training), _abi.ptr(gx), _abi.ptr(gr), _abi.ptr(gw), _abi.ptr(gb),
                  _abi.ptr(gpb), n, c, h, w, ctx.act, _abi.ptr(ws), _abi.dtype_code(gy),
                  _abi.stream_of(gy))
        if want_r and not ctx.act:
            gr = gy
        if want_r and ctx.res_slot is not None:
            # the residual input's other consumer (the block's first conv) adds
            # it in its data-gradient epilogue: no accumulation add (GradSlot)
            ctx.res_slot.put(gr)
            gr = None
        return gx, gw, gb, gpb, gr, None, None, None, None, None, None, None, None, None


def batch_norm_act(x, bn: nn.BatchNorm2d, act: str = "none", residual=None, prebias=None,
                   stats=None, res_slot=None):
    """act(bn(x + prebias) + residual) with nn.BatchNorm2d semantics (mode by bn.training).

    `prebias` is the bias of the convolution feeding this BN, folded in: the
    conv runs without it (no broadcast add, no bias-gradient reduction) and
    its gradient comes out of the BN backward.  `stats` (training only): the
    per-block shifted sums the producing conv's epilogue emitted for x
    (conv3x3_stats / bn_relu_pointwise), replacing the statistics pass.
    `res_slot` (a functional.GradSlot from residual_grad_slot): the residual's
    gradient goes to the slot instead of through autograd.
    """
    _gpu(x, residual, prebias)
    if bn.weight is None or bn.bias is None:
        raise NotImplementedError("affine=False BatchNorm has no HIP kernel")
    training = bn.training or not bn.track_running_stats
    if training and bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm (momentum=None) has no HIP kernel")
    track = bn.training and bn.track_running_stats
    return _BatchNormAct.apply(
        x, bn.weight, bn.bias, prebias, residual,
        bn.running_mean if (track or not training) else None,
        bn.running_var if (track or not training) else None,
        bn.num_batches_tracked if track else None,
        training, bn.momentum if bn.momentum is not None else 0.0, bn.eps, _ACTS[act],
        stats if training else None, res_slot if residual is not None else None)


class _Pointwise(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, x, weight):
        x = x.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        w2 = weight.reshape(cout, cin).contiguous()
        y = torch.empty((n, cout, h, w), dtype=x.dtype, device=x.device)
        _abi.call("mde_pointwise_fwd", _abi.ptr(x), None, None, _abi.ptr(w2), _abi.ptr(y), n, cin,
                  cout, h, w,
                  _abi.dtype_code(x), _abi.stream_of(x))
        ctx.save_for_backward(x, w2)
        ctx.wshape = weight.shape
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        x, w2 = ctx.saved_tensors
        gy = gy.contiguous()
        n, cin, h, w = x.shape
        cout = w2.shape[0]
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw = torch.empty_like(w2)
        ws = _ws(_abi.query("mde_pointwise_workspace", n, cin, cout, h, w), x)
        _abi.call("mde_pointwise_bwd", _abi.ptr(gy), _abi.ptr(x), None, None, _abi.ptr(w2), _abi.ptr(gx),
                  _abi.ptr(gw), n, cin, cout, h, w, _abi.ptr(ws), _abi.dtype_code(gy),
                  _abi.stream_of(gy))
        return gx, gw.view(ctx.wshape)


# mde_pointwise_bwd_bn (the BN backward sums in the 1x1 conv's backward
# epilogue) supports cin <= 32; at cin 64 the separate reduce pass is faster
# (tools/pw_bn_bench.py: 16->8 @480x640 bs32 880 -> 679 us, 32->16 @240x320
# 435 -> ~375 us; 64->32 @120x160 253 vs 264-389 us fused).
_PW_BN_SUMS_MAX_CIN = 32


class _BNReluPointwise(torch.autograd.Function):
    """conv1x1(relu(bn(y1))) with the BN + ReLU applied inside the 1x1 conv's
    operand load: relu(bn(y1)) is never written.  Backward: the 1x1 conv's
    backward recomputes that operand for its weight gradient and returns the
    gradient w.r.t. it; the BN backward (ReLU mask recomputed from y1) turns
    that into d/dy1 and the BN parameter gradients.  A bf16 y1 (autocast:
    the 3x3 conv before ran on MIOpen bf16) stays bf16 -- the kernels read and
    write bf16 activations / gradients with fp32 weights, statistics and
    arithmetic -- so no cast copies surround the fused pair."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, y1, gamma, beta, prebias, running_mean, running_var, nbt, training, momentum,
                eps, w2, stats1=None, want_stats2=False):
        y1 = (y1 if y1.dtype == torch.bfloat16 else y1.float()).contiguous()
        n, c, h, w = y1.shape
        cout = w2.shape[0]
        w2m = w2.reshape(cout, c).contiguous()
        f32 = dict(dtype=torch.float32, device=y1.device)
        scale, shift = torch.empty(c, **f32), torch.empty(c, **f32)
        mean, invstd = torch.empty(c, **f32), torch.empty(c, **f32)
        st = _abi.stream_of(y1)
        ws = _ws(_abi.query("mde_batchnorm_workspace", n, c, h, w), y1) if training else None
        if training and stats1 is not None:  # y1's statistics from the conv3x3 epilogue
            _abi.call("mde_batchnorm_fwd_coef_stats", _abi.ptr(y1), _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(prebias), _abi.ptr(running_mean),
                      _abi.ptr(running_var), _abi.ptr(nbt), float(momentum), float(eps),
                      _abi.ptr(scale), _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(invstd), n, c, h,
                      w, _abi.ptr(stats1), stats1.shape[1], _abi.ptr(ws), _abi.dtype_code(y1), st)
        else:
            _abi.call("mde_batchnorm_fwd_coef", _abi.ptr(y1), _abi.ptr(gamma), _abi.ptr(beta),
                      _abi.ptr(prebias), _abi.ptr(running_mean), _abi.ptr(running_var),
                      _abi.ptr(nbt), float(momentum), float(eps), int(training), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(invstd), n, c, h, w, _abi.ptr(ws),
                      _abi.dtype_code(y1), st)
        y2 = torch.empty((n, cout, h, w), dtype=y1.dtype, device=y1.device)
        if want_stats2:  # y2's statistics for the BatchNorm after this 1x1 conv
            nb = _abi.query("mde_pointwise_stats_blocks", n, c, cout, h, w)
            stats2 = torch.empty((cout, nb, 4), **f32)
            _abi.call("mde_pointwise_fwd_stats", _abi.ptr(y1), _abi.ptr(scale), _abi.ptr(shift),
                      _abi.ptr(w2m), _abi.ptr(y2), _abi.ptr(stats2), n, c, cout, h, w,
                      _abi.dtype_code(y1), st)
        else:
            stats2 = torch.empty((cout, 0, 4), **f32)
            _abi.call("mde_pointwise_fwd", _abi.ptr(y1), _abi.ptr(scale), _abi.ptr(shift),
                      _abi.ptr(w2m), _abi.ptr(y2), n, c, cout, h, w, _abi.dtype_code(y1), st)
        ctx.save_for_backward(y1, gamma, beta, mean, invstd, scale, shift, w2m)
        ctx.training, ctx.has_prebias, ctx.w2shape = bool(training), prebias is not None, w2.shape
        ctx.set_materialize_grads(False)  # no zero-fill launch for the extra output's gradient
        ctx.mark_non_differentiable(stats2)
        return y2, stats2

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy2, _gstats2):
        if gy2 is None:  # only the non-differentiable output was used
            return (None, None, None, None, None, None, None, None, None, None, None, None, None)
        y1, gamma, beta, mean, invstd, scale, shift, w2m = ctx.saved_tensors
        gy2 = gy2.to(y1.dtype).contiguous()
        n, c, h, w = y1.shape
        cout = w2m.shape[0]
        st = _abi.stream_of(gy2)
        gz = torch.empty_like(y1)
        gw2 = torch.empty_like(w2m)
        ws = _ws(_abi.query("mde_pointwise_workspace", n, c, cout, h, w), y1)
        gy1 = torch.empty_like(y1) if ctx.needs_input_grad[0] else None
        gg = torch.empty_like(gamma)
        gb = torch.empty_like(beta)
        gpb = torch.empty_like(gamma) if (ctx.has_prebias and ctx.needs_input_grad[3]) else None
        gy1_out = gy1 if gy1 is not None else torch.empty_like(y1)
        if c <= _PW_BN_SUMS_MAX_CIN:
            # the 1x1 conv's backward also forms the BN backward's two sums in
            # its epilogue, so the BN runs its apply pass only
            sums = torch.empty((c, 2), dtype=torch.float32, device=y1.device)
            _abi.call("mde_pointwise_bwd_bn", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(w2m), _abi.ptr(gz),
                      _abi.ptr(gw2), _abi.ptr(sums), n, c, cout, h, w, _abi.ptr(ws),
                      _abi.dtype_code(gy2), st)
            _abi.call("mde_batchnorm_bwd_apply", _abi.ptr(gz), _abi.ptr(y1), None,
                      _abi.ptr(gamma), _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd),
                      int(ctx.training), _abi.ptr(sums), _abi.ptr(gy1_out), None, _abi.ptr(gg),
                      _abi.ptr(gb), _abi.ptr(gpb), n, c, h, w, _ACTS["relu"],
                      _abi.dtype_code(gy2), st)
        else:
            _abi.call("mde_pointwise_bwd", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(w2m), _abi.ptr(gz), _abi.ptr(gw2), n, c, cout, h,
                      w, _abi.ptr(ws), _abi.dtype_code(gy2), st)
            ws2 = _ws(_abi.query("mde_batchnorm_workspace", n, c, h, w), y1)
            _abi.call("mde_batchnorm_bwd", _abi.ptr(gz), _abi.ptr(y1), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), int(ctx.training),
                      _abi.ptr(gy1_out), None, _abi.ptr(gg), _abi.ptr(gb), _abi.ptr(gpb), n, c,
                      h, w, _ACTS["relu"], _abi.ptr(ws2), _abi.dtype_code(gy2), st)
        return (gy1, gg, gb, gpb, None, None, None, None, None, None, gw2.view(ctx.w2shape), None,
                None)


def bn_relu_pointwise(y1, bn: nn.BatchNorm2d, prebias, conv: nn.Conv2d, stats1=None,
                      want_stats2=False):
    """conv(relu(bn(y1 + prebias))) for a bias-free-folded 1x1 conv on the fused HIP path.

    stats1: y1's per-block statistics from the conv3x3 epilogue (else a
    statistics pass).  Returns (y2, stats2): stats2 is y2's per-block
    statistics for the following BatchNorm when want_stats2, else None."""
    _gpu(y1, prebias)
    if bn.weight is None or bn.bias is None:
        raise NotImplementedError("affine=False BatchNorm has no HIP kernel")
    training = bn.training or not bn.track_running_stats
    if training and bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm (momentum=None) has no HIP kernel")
    track = bn.training and bn.track_running_stats
    y2, stats2 = _BNReluPointwise.apply(
        y1, bn.weight, bn.bias, prebias,
        bn.running_mean if (track or not training) else None,
        bn.running_var if (track or not training) else None,
        bn.num_batches_tracked if track else None,
        training, bn.momentum if bn.momentum is not None else 0.0, bn.eps, conv.weight,
        stats1 if training else None, bool(want_stats2))
    return y2, (stats2 if stats2.shape[1] > 0 else None)


class _SeBnCat(torch.autograd.Function):
    """SELayer(cat([relu(bn_a(ya + pb_a)), relu(bn_b(yb + pb_b))])) from the two
    BatchNorms' raw inputs (mde_se_bn_fwd / _bwd): the BN + ReLU outputs and
    their concatenation are never written, and the backward runs SE, both
    ReLUs and both BatchNorms as one reduction pass + one apply pass."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, ya, yb, ga, ba, pba, gb, bb, pbb, w1, w2, meta_a, meta_b, sta, stb):
        # bf16 storage when either branch is bf16 (autocast; the guide branch's
        # fp32 raw output -- its 3x3 conv on the HIP fp32 kernel -- is rounded,
        # as the reference's bf16 convolution would have produced it)
        dt = torch.bfloat16 if torch.bfloat16 in (ya.dtype, yb.dtype) else torch.float32
        ya, yb = ya.to(dt).contiguous(), yb.to(dt).contiguous()
        w1, w2 = w1.contiguous(), w2.contiguous()
        n, ca, h, w = ya.shape
        cb = yb.shape[1]
        c, cr = ca + cb, w1.shape[0]
        f32 = dict(dtype=torch.float32, device=ya.device)
        scale, shift = torch.empty(c, **f32), torch.empty(c, **f32)
        mean, invstd = torch.empty(c, **f32), torch.empty(c, **f32)
        st = _abi.stream_of(ya)
        for y, g, b, pb, meta, stt, lo, hi in ((ya, ga, ba, pba, meta_a, sta, 0, ca),
                                                (yb, gb, bb, pbb, meta_b, stb, ca, c)):
            rm, rv, nbt, momentum, eps = meta
            cc = hi - lo
            ws = _ws(_abi.query("mde_batchnorm_workspace", n, cc, h, w), y)
            views = [t[lo:hi] for t in (scale, shift, mean, invstd)]
            if stt is not None:
                _abi.call("mde_batchnorm_fwd_coef_stats", _abi.ptr(y), _abi.ptr(g), _abi.ptr(b),
                          _abi.ptr(pb), _abi.ptr(rm), _abi.ptr(rv), _abi.ptr(nbt), float(momentum),
                          float(eps), *[_abi.ptr(v) for v in views], n, cc, h, w, _abi.ptr(stt),
                          stt.shape[1], _abi.ptr(ws), _abi.dtype_code(y), st)
            else:
                _abi.call("mde_batchnorm_fwd_coef", _abi.ptr(y), _abi.ptr(g), _abi.ptr(b),
                          _abi.ptr(pb), _abi.ptr(rm), _abi.ptr(rv), _abi.ptr(nbt), float(momentum),
                          float(eps), 1, *[_abi.ptr(v) for v in views], n, cc, h, w, _abi.ptr(ws),
                          _abi.dtype_code(y), st)
        out = torch.empty((n, c, h, w), dtype=dt, device=ya.device)
        s, hidden, semean = torch.empty((n, c), **f32), torch.empty((n, cr), **f32), torch.empty((n, c), **f32)
        ws = _ws(_abi.query("mde_se_bn_workspace", n, c, cr, h, w), ya)
        _abi.call("mde_se_bn_fwd", _abi.ptr(ya), ca, _abi.ptr(yb), cb, _abi.ptr(scale),
                  _abi.ptr(shift), _abi.ptr(w1), _abi.ptr(w2), cr, _abi.ptr(out), _abi.ptr(s),
                  _abi.ptr(hidden), _abi.ptr(semean), n, h, w, _abi.ptr(ws), _abi.dtype_code(ya), st)
        ctx.save_for_backward(ya, yb, w1, w2, scale, shift, mean, invstd, s, hidden, semean)
        ctx.has_pb = (pba is not None, pbb is not None)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, gout):
        ya, yb, w1, w2, scale, shift, mean, invstd, s, hidden, semean = ctx.saved_tensors
        gout = gout.to(ya.dtype).contiguous()
        n, ca, h, w = ya.shape
        c, cr = ca + yb.shape[1], w1.shape[0]
        gya, gyb = torch.empty_like(ya), torch.empty_like(yb)
        gg, gbt = torch.empty_like(scale), torch.empty_like(scale)
        gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
        ws = _ws(_abi.query("mde_se_bn_workspace", n, c, cr, h, w), ya)
        _abi.call("mde_se_bn_bwd", _abi.ptr(gout), _abi.ptr(ya), ca, _abi.ptr(yb), c - ca,
                  _abi.ptr(scale), _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(invstd), 1,
                  _abi.ptr(w1), _abi.ptr(w2), cr, _abi.ptr(s), _abi.ptr(hidden), _abi.ptr(semean),
                  _abi.ptr(gya), _abi.ptr(gyb), _abi.ptr(gg), _abi.ptr(gbt), _abi.ptr(gw1),
                  _abi.ptr(gw2), n, h, w, _abi.ptr(ws), _abi.dtype_code(gout), _abi.stream_of(gout))
        # a training-mode BatchNorm's output does not depend on its input's
        # per-channel offset: the folded conv biases get zero gradient
        zpa = torch.zeros(ca, dtype=torch.float32, device=ya.device) if ctx.has_pb[0] else None
        zpb = torch.zeros(c - ca, dtype=torch.float32, device=ya.device) if ctx.has_pb[1] else None
        return (gya, gyb, gg[:ca], gbt[:ca], zpa, gg[ca:], gbt[ca:], zpb, gw1, gw2, None, None,
                None, None)


def se_bn_cat(ya, yb, bn_a: nn.BatchNorm2d, bn_b: nn.BatchNorm2d, pb_a, pb_b, w1, w2,
              stats_a=None, stats_b=None):
    """SELayer(cat([relu(bn_a(ya + pb_a)), relu(bn_b(yb + pb_b))], 1)) on the fused
    HIP path (training-mode BatchNorms; fp32, or bf16 storage under autocast).  ya / yb are the raw outputs of
    the 1x1 convs ending feature_conv / guide_conv (modules.py:42-59) and
    stats_a / stats_b their per-block statistics from the conv epilogue (or
    None: a statistics pass).  w1 / w2: SE_block.fc[0] / fc[2] weights."""
    _gpu(ya, yb, pb_a, pb_b, w1, w2)
    for bn in (bn_a, bn_b):
        if bn.weight is None or bn.bias is None or bn.momentum is None or not bn.training:
            raise NotImplementedError("se_bn_cat needs affine, momentum, training-mode BatchNorms")

    def meta(bn):
        track = bn.track_running_stats
        return (bn.running_mean if track else None, bn.running_var if track else None,
                bn.num_batches_tracked if track else None, bn.momentum, bn.eps)

    return _SeBnCat.apply(ya, yb, bn_a.weight, bn_a.bias, pb_a, bn_b.weight, bn_b.bias, pb_b,
                          w1, w2, meta(bn_a), meta(bn_b), stats_a, stats_b)


def pointwise_ok(conv: nn.Conv2d, x) -> bool:
    """Whether this bias-folded 1x1 conv runs on the HIP pointwise kernel."""
    if (conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.padding != (0, 0)
            or conv.dilation != (1, 1) or conv.groups != 1 or x.dim() != 4
            or conv.weight.dtype != torch.float32):
        return False
    return bool(_abi.query("mde_pointwise_supported", conv.in_channels, conv.out_channels,
                           x.shape[2], x.shape[3]))


# Which passes of a bias-free 3x3/s1/p1 conv run on the HIP MFMA kernel
# (mde_conv3x3_*), per (cin, cout): (forward, data gradient, weight gradient).
# The rest go to MIOpen, whose Winograd kernels are faster at >= 32 channels
# (tools/kbench.py --only conv: HIP vs MIOpen per pass at the bench shapes).
# DDRNet's and the decoder's 64/128/256-channel weight gradients run on the
# NCHW wide-channel kernel (cin % 32 == 0, cout % 64 == 0), which needs none
# of MIOpen's NCHW <-> NHWC transposes (tools/wgrad_bench.py);
# MDE_WIDE_WGRAD=0 sends them back to MIOpen (A/B measurement).
CONV3X3_HIP = {
    (3, 16): (True, True, True),
    (3, 32): (True, True, True),
    (3, 64): (True, True, True),
    (16, 16): (True, True, True),
    (32, 32): (False, False, True),
}
WIDE_WGRAD_ALL = os.environ.get("MDE_WIDE_WGRAD", "1") != "0"
WIDE_PAD = os.environ.get("MDE_WIDE_PAD", "1") != "0"  # A/B: 0 = padded shapes on MIOpen
WINO_MIN_BLOCKS = int(os.environ.get("MDE_WINO_MIN_BLOCKS", "256"))  # smallest Winograd grid taken
if WIDE_WGRAD_ALL:
    CONV3X3_HIP.update({(64, 64): (False, False, True), (128, 64): (False, False, True),
                        (128, 128): (False, False, True), (256, 256): (False, False, True)})


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, x, weight, passes, want_stats=False, gx_slot=None):
        wkey = weight  # the Parameter: its Winograd transforms' key in the pack scope
        x = x.contiguous()
        weight = weight.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        stats = torch.empty((cout, 0, 4), dtype=torch.float32, device=x.device)
        ctx.gx_slot = gx_slot
        u_flip = None  # Winograd: the data gradient's filter transform, made with the forward's
        if passes[0] == WINO:  # Winograd F(2x2, 3x3) (wino.hip), + the BN statistics
            y = torch.empty((n, cout, h, w), dtype=x.dtype, device=x.device)
            st = _abi.stream_of(x)
            if want_stats:
                nb = _abi.query("mde_wino_stats_blocks", n, cin, cout, h, w)
                stats = torch.empty((cout, nb, 4), dtype=torch.float32, device=x.device)
            flip = passes[1] == WINO  # the data gradient's flipped transform too
            sc = _ACTIVE_PACK
            ent = sc.wino.get(wkey) if sc is not None else None
            if ent is not None and wkey in sc.wino_packed and (ent[1] is not None or not flip):
                u, u_flip = ent[0], (ent[1] if flip else None)  # made by the scope's table launch
            else:
                ub = _abi.query("mde_wino_weight_bytes", cin, cout) // 4  # padded channels included
                u = torch.empty(ub, dtype=torch.float32, device=x.device)
                if flip:  # both transforms in one launch
                    u_flip = torch.empty(ub, dtype=torch.float32, device=x.device)
                    _abi.call("mde_wino_weight2", _abi.ptr(weight), _abi.ptr(u), _abi.ptr(u_flip),
                              cin, cout, st)
                else:
                    _abi.call("mde_wino_weight", _abi.ptr(weight), _abi.ptr(u), cin, cout, 0, st)
                if (sc is not None and ent is None and isinstance(wkey, nn.Parameter)
                        and not torch.cuda.is_current_stream_capturing()):
                    sc.wino[wkey] = (u, u_flip, cin, cout)  # in the table from the next forward
            _abi.call("mde_wino_conv_stats", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y),
                      _abi.ptr(stats) if want_stats else None, n, cin, cout, h, w, 0,
                      _abi.dtype_code(x), st)
        elif passes[0] == WIDE:  # no statistics epilogue: the BatchNorm reads y
            y = torch.empty((n, cout, h, w), dtype=x.dtype, device=x.device)
            _abi.call("mde_conv3x3_wide_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cin,
                      cout, h, w, _abi.dtype_code(x), _abi.stream_of(x))
        elif passes[0]:
            y = torch.empty((n, cout, h, w), dtype=x.dtype, device=x.device)
            if want_stats:  # + y's per-block BN statistics from the epilogue
                nb = _abi.query("mde_conv3x3_stats_blocks", n, cin, cout, h, w, _abi.MDE_F32)
                stats = torch.empty((cout, nb, 4), dtype=torch.float32, device=x.device)
                _abi.call("mde_conv3x3_fwd_stats", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y),
                          _abi.ptr(stats), n, cin, cout, h, w, _abi.dtype_code(x),
                          _abi.stream_of(x))
            else:
                _abi.call("mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cin,
                          cout, h, w, _abi.dtype_code(x), _abi.stream_of(x))
        else:
            y = torch.nn.functional.conv2d(x, weight, None, 1, 1)
        ctx.save_for_backward(x, weight)
        ctx.passes = passes
        ctx.u_flip = u_flip
        ctx.set_materialize_grads(False)  # no zero-fill launch for the extra output's gradient
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy, _gstats):
        # the residual path's gradient of x, handed over by the BatchNorm that
        # adds x back (residual_grad_slot): summed into gx here
        g2 = ctx.gx_slot.take() if ctx.gx_slot is not None else None
        if gy is None:  # only the non-differentiable output was used
            return (g2, None, None, None, None)
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        gx = gw = None
        st = _abi.stream_of(gy)
        if ctx.needs_input_grad[0]:
            if ctx.passes[1] == WINO:  # the flipped, transposed filter's transform
                gx = torch.empty_like(x)
                u = ctx.u_flip
                if u is None:
                    u = torch.empty(_abi.query("mde_wino_weight_bytes", cin, cout) // 4,
                                    dtype=torch.float32, device=x.device)
                    _abi.call("mde_wino_weight", _abi.ptr(weight), _abi.ptr(u), cin, cout, 1, st)
                if g2 is not None and g2.dtype == gy.dtype == torch.float32:
                    g2 = g2.contiguous()  # held until the launch is enqueued
                    _abi.call("mde_wino_conv_acc", _abi.ptr(gy), _abi.ptr(u), _abi.ptr(g2),
                              _abi.ptr(gx), n, cout, cin, h, w, 1, _abi.dtype_code(gy), st)
                    g2 = None
                else:
                    _abi.call("mde_wino_conv", _abi.ptr(gy), _abi.ptr(u), _abi.ptr(gx), n, cout,
                              cin, h, w, 1, _abi.dtype_code(gy), st)
            elif ctx.passes[1] == WIDE:
                gx = torch.empty_like(x)
                _abi.call("mde_conv3x3_wide_bwd_data", _abi.ptr(gy), _abi.ptr(weight), _abi.ptr(gx),
                          n, cin, cout, h, w, _abi.dtype_code(gy), st)
            elif ctx.passes[1]:
                gx = torch.empty_like(x)
                _abi.call("mde_conv3x3_bwd_data", _abi.ptr(gy), _abi.ptr(weight), _abi.ptr(gx), n,
                          cin, cout, h, w, _abi.dtype_code(gy), st)
            else:
                # MIOpen data gradient; the saved x stands in for the input
                # (torch.nn.grad.conv2d_input passes an expanded dummy, which
                # the backend materialises: a full-size copy per call)
                gx = torch.ops.aten.convolution_backward(
                    gy, x, weight, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                    (True, False, False))[0]
        if ctx.needs_input_grad[1]:
            if ctx.passes[2]:
                gw = torch.empty_like(weight)
                ws = _ws(_abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w,
                                    _abi.MDE_F32), x)
                _abi.call("mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin,
                          cout, h, w, _abi.ptr(ws), _abi.dtype_code(gy), st)
            else:
                gw = torch.ops.aten.convolution_backward(
                    gy, x, weight, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                    (False, True, False))[1]
        if g2 is not None:  # a data-gradient kernel with no accumulating epilogue
            gx = g2 if gx is None else gx + g2
        return gx, gw, None, None, None


# bf16 (autocast) 3x3 convolutions on the v_mfma_f32_16x16x32_bf16 kernels:
# (cin, cout) -> (fwd, dgrad, wgrad).  The 3-channel guide convolutions read
# the fp32 image and stay on the fp32 kernels.
CONV3X3_HIP_BF16 = {
    (16, 16): (True, True, True),
    (32, 32): (True, True, True),
}
if os.environ.get("MDE_C3BF32", "1") == "0":  # A/B: 32 -> 32 on convbf.hip instead
    del CONV3X3_HIP_BF16[(32, 32)]


def _autocast_bf16(x) -> bool:
    return (x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16)


def _conv3x3_bf16_path(cin: int, cout: int, x, weight) -> bool:
    """autocast-bf16 (or bf16) input of a shape the bf16 kernels take.  The
    kernels read an fp32 weight (rounded to bf16 on load) and write an fp32
    weight gradient: a weight of any other dtype never takes them."""
    return ((_autocast_bf16(x) or x.dtype == torch.bfloat16)
            and weight.dtype == torch.float32
            and (cin, cout) in CONV3X3_HIP_BF16 and x.shape[-1] % 4 == 0)


class _Conv3x3Bf16(torch.autograd.Function):
    """The bf16 autocast 3x3 convolution (16 -> 16, 32 -> 32) on
    v_mfma_f32_16x16x32_bf16: x / y / gx bf16, the fp32 weight rounded to
    bf16 inside the kernels (as autocast's cast), fp32 accumulation, fp32
    weight gradient.  Passes with a False flag run on MIOpen's bf16 kernels."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, x, weight, passes, want_stats=False):
        x = x.contiguous()
        weight = weight.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        bf = _abi.MDE_BF16
        stats = torch.empty((cout, 0, 4), dtype=torch.float32, device=x.device)
        if passes[0]:
            y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device)
            if want_stats:
                nb = _abi.query("mde_conv3x3_stats_blocks", n, cin, cout, h, w, bf)
                stats = torch.empty((cout, nb, 4), dtype=torch.float32, device=x.device)
                _abi.call("mde_conv3x3_fwd_stats", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y),
                          _abi.ptr(stats), n, cin, cout, h, w, bf, _abi.stream_of(x))
            else:
                _abi.call("mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cin,
                          cout, h, w, bf, _abi.stream_of(x))
        else:
            y = torch.nn.functional.conv2d(x, weight.to(torch.bfloat16), None, 1, 1)
        ctx.save_for_backward(x, weight)
        ctx.passes = passes
        ctx.set_materialize_grads(False)  # no zero-fill launch for the extra output's gradient
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy, _gstats):
        if gy is None:  # only the non-differentiable output was used
            return (None, None, None, None)
        x, weight = ctx.saved_tensors
        gy = gy.to(torch.bfloat16).contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        bf = _abi.MDE_BF16
        gx = gw = None
        st = _abi.stream_of(gy)
        if ctx.needs_input_grad[0]:
            if ctx.passes[1]:
                gx = torch.empty_like(x)
                _abi.call("mde_conv3x3_bwd_data", _abi.ptr(gy), _abi.ptr(weight), _abi.ptr(gx), n,
                          cin, cout, h, w, bf, st)
            else:
                gx = torch.ops.aten.convolution_backward(
                    gy, x, weight.to(torch.bfloat16), None, (1, 1), (1, 1), (1, 1), False, (0, 0),
                    1, (True, False, False))[0]
        if ctx.needs_input_grad[1]:
            if ctx.passes[2]:
                gw = torch.empty_like(weight)
                ws = _ws(_abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w, bf), x)
                _abi.call("mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin,
                          cout, h, w, _abi.ptr(ws), bf, st)
            else:
                gw = torch.ops.aten.convolution_backward(
                    gy, x, weight.to(torch.bfloat16), None, (1, 1), (1, 1), (1, 1), False, (0, 0),
                    1, (False, True, False))[1].float()
        return gx, gw, None, None


class _Conv3x3S2(torch.autograd.Function):
    """Bias-free k3 / s2 / p1 convolution (DDRNet's stem convs, the stride-2
    BasicBlock convs, down3 / down4, layer5's Bottleneck conv2:
    DDRNet_23_slim.py:41-72,80,232-233,254-265): the weight gradient on the HIP
    stride-2 kernel (mde_conv3x3s2_wgrad), the forward and data gradient on
    the HIP MFMA kernels of conv3x3s2.hip where a shape has one (>= 32
    channels; MDE_S2_FWD=0: MIOpen), else MIOpen -- all NCHW, no NHWC
    transposes on the HIP passes."""

    @staticmethod
    def forward(ctx, x, weight):
        x = x.contiguous()
        weight = weight.contiguous()
        ctx.save_for_backward(x, weight)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        if S2_FWD and _abi.query("mde_conv3x3s2_fwd_supported", cin, cout, h, w, _abi.MDE_F32):
            y = torch.empty((n, cout, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=x.dtype,
                            device=x.device)
            _abi.call("mde_conv3x3s2_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cin, cout,
                      h, w, _abi.dtype_code(x), _abi.stream_of(x))
            return y
        return torch.nn.functional.conv2d(x, weight, None, 2, 1)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        gx = gw = None
        if ctx.needs_input_grad[0]:
            if S2_FWD and _abi.query("mde_conv3x3s2_dgrad_supported", cin, cout, h, w,
                                     _abi.MDE_F32):
                gx = torch.empty_like(x)
                _abi.call("mde_conv3x3s2_bwd_data", _abi.ptr(gy), _abi.ptr(weight), _abi.ptr(gx), n,
                          cin, cout, h, w, _abi.dtype_code(gy), _abi.stream_of(gy))
            else:
                gx = torch.ops.aten.convolution_backward(
                    gy, x, weight, None, (2, 2), (1, 1), (1, 1), False, (0, 0), 1,
                    (True, False, False))[0]
        if ctx.needs_input_grad[1]:
            nws = _abi.query("mde_conv3x3s2_wgrad_workspace", n, cin, cout, h, w, _abi.MDE_F32) \
                if (S2_WGRAD and (S2_WIDE or cout == 32)
                    and _abi.query("mde_conv3x3s2_supported", cin, cout, _abi.MDE_F32)) else 0
            if nws > 0:
                gw = torch.empty_like(weight)
                _abi.call("mde_conv3x3s2_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin,
                          cout, h, w, _abi.ptr(_ws(nws, x)), _abi.MDE_F32, _abi.stream_of(gy))
            else:
                gw = torch.ops.aten.convolution_backward(
                    gy, x, weight, None, (2, 2), (1, 1), (1, 1), False, (0, 0), 1,
                    (False, True, False))[1]
        return gx, gw


class _Conv1x1(torch.autograd.Function):
    """Bias-free wide 1x1 convolution, stride 1 or 2 (DDRNet's Bottleneck /
    downsample / compression / DAPPM convs, DDRNet_23_slim.py:79,84,121-171,
    245,250,294-296): forward, data gradient and weight gradient on the NCHW
    MFMA kernels of conv1x1.hip (no NHWC transposes)."""

    @staticmethod
    def forward(ctx, x, weight, stride):
        x = x.contiguous()
        weight = weight.contiguous()
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        cin, cout = x.shape[1], weight.shape[0]
        if stride == 1 and not (C1_FWD == "all" or (C1_FWD == "pad" and (cin % 32 or cout % 32))):
            # MIOpen runs the stride-1 forward as one NCHW GEMM (rocBLAS, no
            # transposes), as fast or faster than the HIP kernel at DDRNet's
            # shapes (tools/c1_bench.py): only its backward needs replacing.
            # Channel counts off the 32 grid (MobileNetV3's) take the HIP
            # forward: MIOpen picks its Winograd / NHWC solvers there
            return torch.nn.functional.conv2d(x, weight)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
        y = torch.empty((n, cout, ho, wo), dtype=x.dtype, device=x.device)
        _abi.call("mde_conv1x1_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cin, cout, h, w,
                  stride, _abi.dtype_code(x), _abi.stream_of(x))
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        st = _abi.stream_of(gy)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _abi.call("mde_conv1x1_bwd_data", _abi.ptr(gy), _abi.ptr(weight), _abi.ptr(gx), n, cin,
                      cout, h, w, ctx.stride, _abi.dtype_code(gy), st)
        if ctx.needs_input_grad[1]:
            gw = torch.empty_like(weight)
            ws = _ws(_abi.query("mde_conv1x1_wgrad_workspace", n, cin, cout, h, w, ctx.stride,
                                _abi.MDE_F32), x)
            _abi.call("mde_conv1x1_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin, cout, h,
                      w, ctx.stride, _abi.ptr(ws), _abi.dtype_code(gy), st)
        return gx, gw, None


C1_WIDE = os.environ.get("MDE_C1_WIDE", "1") != "0"  # MDE_C1_WIDE=0: MIOpen (A/B switch)
C1_PAD = os.environ.get("MDE_C1_PAD", "1") != "0"  # A/B: 0 = only channel counts % 32 (round 5)
C1_FWD = os.environ.get("MDE_C1_FWD", "pad")  # stride-1 HIP forward: pad (off-grid channels) / all / none


def conv1x1_ok(conv: nn.Conv2d, x) -> bool:
    """Whether this bias-free 1x1 conv (stride 1 or 2) runs on the wide HIP 1x1
    kernels: fp32 outside autocast, channel counts multiples of 8 and >= 16
    (padded to 32 in-kernel; MobileNetV3's expand / project convs); the
    small-channel decoder 1x1s keep the fused pointwise kernels."""
    if not (C1_WIDE and x.is_cuda and x.dtype == torch.float32 and not _autocast_bf16(x)
            and conv.weight.dtype == torch.float32 and x.dim() == 4
            and conv.kernel_size == (1, 1) and conv.padding == (0, 0)
            and conv.dilation == (1, 1) and conv.groups == 1
            and conv.stride in ((1, 1), (2, 2)) and conv.padding_mode == "zeros"):
        return False
    if not C1_PAD and (conv.in_channels % 32 or conv.out_channels % 32):
        return False
    return bool(_abi.query("mde_conv1x1_supported", conv.in_channels, conv.out_channels,
                           x.shape[2], x.shape[3], conv.stride[0], _abi.MDE_F32))


def conv3x3s2_ok(conv: nn.Conv2d, x) -> bool:
    """Whether this k3 / s2 / p1 conv takes _Conv3x3S2: fp32 outside autocast,
    even input width, and a HIP kernel for at least one pass -- the stride-2
    weight gradient (the stem's 3 -> 32 / 32 -> 32, 32+ -> 64+ channels at
    output widths that are multiples of 40 or 20; MDE_S2_WGRAD=0: MIOpen) or
    the forward / data gradient (>= 32 channels, conv3x3s2.hip; MDE_S2_FWD=0:
    MIOpen).  The passes without one run on MIOpen inside the Function."""
    if not (x.is_cuda and x.dtype == torch.float32 and not _autocast_bf16(x)
            and conv.weight.dtype == torch.float32 and x.dim() == 4 and x.shape[-1] % 2 == 0
            and conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.padding_mode == "zeros"):
        return False
    cin, cout, h, w = conv.in_channels, conv.out_channels, x.shape[2], x.shape[3]
    wgrad = (S2_WGRAD and bool(_abi.query("mde_conv3x3s2_supported", cin, cout, _abi.MDE_F32))
             and (S2_WIDE or cout == 32)
             and _abi.query("mde_conv3x3s2_wgrad_workspace", x.shape[0], cin, cout, h, w,
                            _abi.MDE_F32) > 0)
    fwd = S2_FWD and bool(_abi.query("mde_conv3x3s2_fwd_supported", cin, cout, h, w, _abi.MDE_F32))
    return wgrad or fwd


S2_WGRAD = os.environ.get("MDE_S2_WGRAD", "1") != "0"
S2_FWD = os.environ.get("MDE_S2_FWD", "1") != "0"  # HIP stride-2 forward / data gradient (A/B switch)
S2_WIDE = os.environ.get("MDE_S2_WIDE", "1") != "0"  # the 64+-channel ones (A/B switch)


def conv3x3_passes(conv: nn.Conv2d, x):
    """(fwd, dgrad, wgrad) HIP flags for a 3x3/s1/p1 conv, or None if it is not one.

    Under bf16 autocast the 16 -> 16 / 32 -> 32 convs run on the bf16 MFMA
    kernels (autocast's conv semantics: bf16 operands, fp32 accumulation,
    bf16 output, no NCHW <-> NHWC transposes); other bf16 inputs go to
    MIOpen's bf16 kernels; fp32 inputs (also the guide convs' image under
    autocast) to the fp32 kernels."""
    if (conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1)
            or conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros"
            or x.dim() != 4 or conv.weight.dtype != torch.float32):
        return None  # the HIP kernels take an fp32 weight only (bf16 modules: MIOpen)
    cin, cout = conv.in_channels, conv.out_channels
    if _conv3x3_bf16_path(cin, cout, x, conv.weight):
        p, dt = CONV3X3_HIP_BF16[(cin, cout)], _abi.MDE_BF16
    elif x.dtype == torch.float32:
        p, dt = CONV3X3_HIP.get((cin, cout), (False, False, False)), _abi.MDE_F32
    else:
        return None
    p = [bool(f) and bool(_abi.query("mde_conv3x3_supported", cin, cout, i, dt))
         for i, f in enumerate(p)]
    if (dt == _abi.MDE_F32 and WIDE_WGRAD_ALL and not p[2] and cout % 64 == 0
            and _abi.query("mde_conv3x3_supported", cin, cout, 2, dt)
            and (cin % 32 == 0 or (WIDE_PAD and _abi.query(
                "mde_conv3x3_wgrad_workspace", x.shape[0], cin, cout, x.shape[2], x.shape[3],
                dt)))):
        # any other wide-channel weight gradient (the NewCRF projections,
        # newcrf_layers.py:384-392,420-423: 64-1024 channels) on the NCHW HIP
        # kernel: per shape it matches MIOpen's NHWC implicit GEMM, and the
        # NCHW <-> NHWC transposes around that one disappear; (round 6) also
        # 24 / 40 / 112 input channels, padded to the next 32 (where MIOpen
        # ran its Winograd weight gradient, miopenSp3AsmConv f3x2)
        p[2] = True
    if dt == _abi.MDE_F32 and WINO_ON and not _autocast_bf16(x):
        # forward / data gradient of the 32-256-channel convs on the Winograd
        # F(2x2, 3x3) kernels (2.25x fewer MACs) where MIOpen would run its own
        # Winograd: 64- / 32-channel output groups (the 16-channel variant
        # loses to the direct kernel: the input transform is amortised over
        # too few output channels, tools/wino_bench.py) on planes of >= 256
        # blocks (8 x 16 output pixels x 64 / 32 channels)
        # (round 6) channel counts off the 16 / 32 grid too -- the NewCRF
        # projections proj_x 24 -> 128, 40 -> 256 and the data gradients into
        # 24 / 40 / 112 channels, newcrf_layers.py:384-392 -- with padded
        # channels (wino.hip wino_geo: zero planes / filter rows, unstored
        # outputs), where MIOpen's Winograd and its NHWC transposes ran
        n, h, w = x.shape[0], x.shape[2], x.shape[3]
        for i, (a, b) in enumerate(((cin, cout), (cout, cin))):
            bp = b if b == 16 else -(-b // 32) * 32  # output channels as padded
            blocks = n * -(-h // 8) * -(-w // 16) * (bp // (64 if bp % 64 == 0 else 32))
            aligned = b % (32 if WINO32 else 64) == 0 and a % 16 == 0
            if (not p[i] and (aligned or (WINO_PAD and b > 16)) and blocks >= WINO_MIN_BLOCKS
                    and _abi.query("mde_wino_supported", a, b, h, w, _abi.MDE_F32)):
                p[i] = WINO
    if dt == _abi.MDE_F32 and C3_WIDE and not _autocast_bf16(x):
        # forward / data gradient of the 32-256-channel convs on the band-GEMM
        # kernels (conv3x3s2.hip c3s1_kernel) where MIOpen would run Winograd
        for i in (0, 1):
            if not p[i] and _abi.query("mde_conv3x3_wide_supported", cin, cout, x.shape[2],
                                       x.shape[3], i, dt):
                p[i] = WIDE
    return tuple(p) if any(p) else None


WIDE = 2  # conv3x3_passes flag: the pass runs on the wide-channel kernel
WINO = 3  # conv3x3_passes flag: the pass runs on the Winograd kernel
# MDE_WINO=0: MIOpen for these passes (A/B switch; cfg2 interleaved A/B 911.6 /
# 909.0 vs 881.0 / 878.3 img/s, profiles/r04_ab_wino.txt)
WINO_ON = os.environ.get("MDE_WINO", "1") != "0"
WINO32 = os.environ.get("MDE_WINO32", "1") != "0"  # the 32-channel output groups too (A/B)
WINO_PAD = os.environ.get("MDE_WINO_PAD", "1") != "0"  # padded channel counts too (A/B)
# Off by default: MIOpen's Winograd matches the stride-1 band kernel on these
# shapes (tools/c1_bench.py) and the cfg2 step was 0.5 % slower with it on
C3_WIDE = os.environ.get("MDE_C3_WIDE", "0") == "1"


class _PackScope:
    """The bf16 filters of one model's convbf convolutions, packed for a whole
    forward in ONE launch (mde_convbf_pack_table) when the model's forward
    enters convbf_pack_scope, instead of one pack launch per conv (48 a cfg3
    step, ~7 us each).  A conv is registered on its first eager forward (its
    persistent packed buffers allocated then) and is in the table from the
    next forward; inside a graph capture nothing is registered or rebuilt, so
    the captured launch packs the table of the last eager step."""

    def __init__(self):
        self.entries = {}  # weight -> (packed, packed_t, cin, cout, ks)
        self.table = None
        self.retired = []  # earlier tables, kept alive for the graphs that captured them
        self.rows = []  # weights in table order
        self.ptrs = ()
        self.blocks = 0
        self.elems = 0
        self.packed = frozenset()  # weights packed by this forward's table launch
        # the fp32 Winograd convs' filter transforms (wino.hip), the same way:
        # weight -> (U, U' or None, cin, cout), one mde_wino_weight_table launch
        # (the per-conv mde_wino_weight2 launches: 27 a cfg2 step)
        self.wino = {}
        self.wtable = None
        self.wrows = []
        self.wptrs = ()
        self.wblocks = 0
        self.wpairs = 0
        self.wino_packed = frozenset()

    def _ptrs(self):
        return tuple(w.data_ptr() for w in self.entries)

    def refresh(self, device):
        """Rebuild the device table when convs were registered or a weight moved."""
        ptrs = self._ptrs()
        if self.table is not None and ptrs == self.ptrs:
            return
        rows, blk, elems = [], 0, 0
        for wgt, (wp, wt, cin, cout, ks) in self.entries.items():
            rows.append([wgt.data_ptr(), wp.data_ptr(), wt.data_ptr(), cin, cout, ks, blk, 0])
            blk += -(-max(wp.numel(), wt.numel()) // 256)
            elems += wp.numel() + wt.numel()
        if self.table is not None:
            # a captured step graph recorded this table's device pointer in its
            # pack node (and reads the weight / packed pointers it holds): never
            # free a table a graph may still replay
            self.retired.append(self.table)
        self.table = torch.tensor(rows, dtype=torch.int64, device=device)
        self.rows, self.ptrs, self.blocks, self.elems = list(self.entries), ptrs, blk, elems

    def refresh_wino(self, device):
        """The Winograd table (rows: weight, U, U' or 0, cin, cout, first block)."""
        ptrs = tuple(w.data_ptr() for w in self.wino)
        if self.wtable is not None and ptrs == self.wptrs:
            return
        rows, blk, pairs = [], 0, 0
        for wgt, (u, uf, cin, cout) in self.wino.items():
            rows.append([wgt.data_ptr(), u.data_ptr(), uf.data_ptr() if uf is not None else 0,
                         cin, cout, blk, 0, 0])
            blk += _abi.query("mde_wino_weight_blocks", cin, cout, int(uf is not None))
            pairs += cin * cout
        if self.wtable is not None:
            self.retired.append(self.wtable)  # a captured graph may still read it
        self.wtable = torch.tensor(rows, dtype=torch.int64, device=device)
        self.wrows, self.wptrs, self.wblocks, self.wpairs = list(self.wino), ptrs, blk, pairs


CONVBF_PACK_ALL = os.environ.get("MDE_CONVBF_PACK_ALL", "1") != "0"  # A/B: 0 = a pack per conv
WINO_TABLE = os.environ.get("MDE_WINO_TABLE", "1") != "0"  # A/B: 0 = a transform launch per conv
_ACTIVE_PACK = None


@contextlib.contextmanager
def convbf_pack_scope(owner: nn.Module, device):
    """Run `owner`'s forward with its registered convbf filters packed by one
    launch at entry, and its registered fp32 Winograd filter transforms made
    by one more (see _PackScope); a no-op off the GPU or with
    MDE_CONVBF_PACK_ALL=0 (MDE_WINO_TABLE=0: the Winograd launch per conv)."""
    global _ACTIVE_PACK
    if not (CONVBF_PACK_ALL and device.type == "cuda" and _ACTIVE_PACK is None):
        yield
        return
    sc = owner.__dict__.get("_convbf_pack")
    if sc is None:
        sc = owner.__dict__["_convbf_pack"] = _PackScope()
    capturing = torch.cuda.is_current_stream_capturing()
    if sc.entries and not capturing:
        sc.refresh(device)
    if sc.wino and not capturing:
        sc.refresh_wino(device)
    sc.packed = frozenset()
    sc.wino_packed = frozenset()
    if sc.table is not None:
        _abi.call("mde_convbf_pack_table", _abi.ptr(sc.table), len(sc.rows), sc.blocks, sc.elems,
                  _abi.stream_of(sc.table))
        sc.packed = frozenset(sc.rows)
    if sc.wtable is not None and WINO_TABLE:
        _abi.call("mde_wino_weight_table", _abi.ptr(sc.wtable), len(sc.wrows), sc.wblocks,
                  sc.wpairs, _abi.stream_of(sc.wtable))
        sc.wino_packed = frozenset(sc.wrows)
    _ACTIVE_PACK = sc
    try:
        yield
    finally:
        _ACTIVE_PACK = None


class _ConvBf16(torch.autograd.Function):
    """A DDRNet convolution under bf16 autocast (3x3 p1 / 1x1 p0, stride 1 or
    2, channels % 32) on the bf16 implicit-GEMM kernels of convbf.hip:
    autocast's conv semantics -- x cast to bf16, the fp32 weight rounded to
    bf16, fp32 accumulation, bf16 y / gx, fp32 weight gradient -- in NCHW,
    with none of MIOpen's NHWC transposes or cast / zero-fill kernels.  Both
    packed filters (forward; transposed for the data gradient) come from one
    launch in the forward.  want_stats: the following BatchNorm's per-block
    statistics of y from the forward's epilogue (else an empty tensor).
    DDRNet_23_slim.py:35-38,41-113,121-171,230-263 (every conv of the encoder
    but the 3-channel stem)."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, x, weight, ks, stride, want_stats):
        x = x.to(torch.bfloat16).contiguous()
        weight = weight.contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        pad = ks // 2
        ho, wo = (h + 2 * pad - ks) // stride + 1, (w + 2 * pad - ks) // stride + 1
        st = _abi.stream_of(x)
        bf = dict(dtype=torch.bfloat16, device=x.device)
        sc = _ACTIVE_PACK
        ent = sc.entries.get(weight) if sc is not None else None
        if ent is not None and weight in sc.packed:
            wp, wt = ent[0], ent[1]  # packed at the scope's entry with every other filter
        else:
            wp = torch.empty(_abi.query("mde_convbf_pack_elems", cin, cout, ks, 0), **bf)
            wt = torch.empty(_abi.query("mde_convbf_pack_elems", cin, cout, ks, 1), **bf)
            _abi.call("mde_convbf_pack_both", _abi.ptr(weight), _abi.ptr(wp), _abi.ptr(wt), cin,
                      cout, ks, st)
            if (sc is not None and ent is None and isinstance(weight, nn.Parameter)
                    and not torch.cuda.is_current_stream_capturing()):
                sc.entries[weight] = (wp, wt, cin, cout, ks)  # in the table from the next forward
                sc.dirty = True
        y = torch.empty((n, cout, ho, wo), **bf)
        nb = _abi.query("mde_convbf_stats_blocks", n, cin, cout, h, w, ks, stride) if want_stats else 0
        stats = torch.empty((cout, nb, 4), dtype=torch.float32, device=x.device)
        _abi.call("mde_convbf_fwd", _abi.ptr(x), _abi.ptr(wp), _abi.ptr(y),
                  _abi.ptr(stats) if nb else None, n, cin, cout, h, w, ks, stride, st)
        ctx.save_for_backward(x, weight, wt)
        ctx.ks, ctx.stride = ks, stride
        ctx.set_materialize_grads(False)  # no zero-fill launch for the statistics' gradient
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy, _gstats):
        if gy is None:
            return None, None, None, None, None
        x, weight, wt = ctx.saved_tensors
        gy = gy.to(torch.bfloat16).contiguous()
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        ks, stride = ctx.ks, ctx.stride
        st = _abi.stream_of(gy)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _abi.call("mde_convbf_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, cin, cout,
                      h, w, ks, stride, st)
        if ctx.needs_input_grad[1]:
            gw = torch.empty_like(weight)
            ws = _ws(_abi.query("mde_convbf_wgrad_workspace", n, cin, cout, h, w, ks, stride), x)
            _abi.call("mde_convbf_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin, cout, h, w,
                      ks, stride, _abi.ptr(ws), st)
        return gx, gw, None, None, None


class _StemBf16(torch.autograd.Function):
    """DDRNet's stem conv (3 -> 32, 3x3, stride 2, padding 1; DDRNet_23_slim.py:
    230-233) under bf16 autocast on stem.hip: the fp32 image and weight rounded
    to bf16 in the kernels (autocast's casts), fp32 accumulation, a bf16
    output, the fp32 weight gradient; the image takes no gradient.  Replaces
    MIOpen's NHWC bf16 solvers, their transposes and zero fills."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, x, weight):
        x = x.contiguous()
        weight = weight.contiguous()
        n, _, h, w = x.shape
        cout = weight.shape[0]
        y = torch.empty((n, cout, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=torch.bfloat16,
                        device=x.device)
        _abi.call("mde_stem_bf16_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, cout, h, w,
                  _abi.stream_of(x))
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gw = None
        if ctx.needs_input_grad[1]:
            gy = gy.to(torch.bfloat16).contiguous()
            n, _, h, w = x.shape
            cout = weight.shape[0]
            gw = torch.empty_like(weight)
            ws = _ws(_abi.query("mde_stem_bf16_wgrad_workspace", n, cout, h, w), x)
            _abi.call("mde_stem_bf16_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cout, h, w,
                      _abi.ptr(ws), _abi.stream_of(gy))
        return None, gw


STEM_BF16 = os.environ.get("MDE_STEM_BF16", "1") != "0"  # A/B switch: 0 = MIOpen


def stem_ok(conv: nn.Conv2d, x) -> bool:
    """Whether this conv takes _StemBf16: an fp32 CUDA image that needs no
    gradient under bf16 autocast, 3 -> 32 / 64 channels, 3x3 / stride 2 /
    padding 1, zero padding, width % 4 == 0."""
    return (STEM_BF16 and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
            and not x.requires_grad and _autocast_bf16(x) and conv.weight.dtype == torch.float32
            and conv.in_channels == 3 and conv.kernel_size == (3, 3) and conv.stride == (2, 2)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.padding_mode == "zeros"
            and x.numel() < (1 << 31)  # the kernels' 32-bit image offsets (n*3*h*w)
            and bool(_abi.query("mde_stem_bf16_supported", 3, conv.out_channels, x.shape[2],
                                x.shape[3])))


CONVBF = os.environ.get("MDE_CONVBF", "1") != "0"  # A/B switch: 0 = MIOpen's bf16 solvers
_CONVBF_OK: dict = {}


def convbf_ok(conv: nn.Conv2d, x) -> bool:
    """Whether this conv runs on convbf.hip: a CUDA input under bf16 autocast
    (or already bf16), fp32 weight, 3x3 / padding 1 or 1x1 / padding 0,
    stride 1 or 2, zero padding, no groups / dilation, and all three passes
    supported for the shape (channels % 32, even width, LDS capacity)."""
    if not (CONVBF and x.is_cuda and x.dim() == 4
            and (_autocast_bf16(x) or x.dtype == torch.bfloat16)
            and conv.weight.dtype == torch.float32 and conv.groups == 1
            and conv.dilation == (1, 1) and conv.padding_mode == "zeros"
            and conv.stride in ((1, 1), (2, 2))
            and ((conv.kernel_size == (3, 3) and conv.padding == (1, 1))
                 or (conv.kernel_size == (1, 1) and conv.padding == (0, 0)))):
        return False
    # the real batch: a launch refuses n x patches >= 2^22, which the batch-free
    # query cannot see -- such a batch falls back to MIOpen here instead of
    # raising inside the step
    key = (x.shape[0], conv.in_channels, conv.out_channels, x.shape[2], x.shape[3],
           conv.kernel_size[0], conv.stride[0])
    ok = _CONVBF_OK.get(key)
    if ok is None:
        ok = all(_abi.query("mde_convbf_supported_n", *key, p) for p in (0, 1, 2))
        _CONVBF_OK[key] = ok
    return ok


def conv_bf16(conv: nn.Conv2d, x):
    """conv(x) without its bias on convbf.hip (see convbf_ok)."""
    _gpu(x)
    return _ConvBf16.apply(x, conv.weight, conv.kernel_size[0], conv.stride[0], False)[0]


def conv_bf16_stats(conv: nn.Conv2d, x):
    """conv_bf16 that also returns y's per-block BN statistics [cout][blocks][4]
    (shift, count, s1, s2) from the forward epilogue."""
    _gpu(x)
    y, stats = _ConvBf16.apply(x, conv.weight, conv.kernel_size[0], conv.stride[0], True)
    return y, (stats if stats.shape[1] > 0 else None)


class _GuideConvBf16(torch.autograd.Function):
    """The guided-upsampling blocks' guide convs (3 -> 16 / 32 / 64 on the
    image, modules.py:52-54) under bf16 autocast: the fp32 image and weight
    rounded to bf16 in the kernel (autocast's casts), fp32 accumulation, a
    bf16 output (mde_conv3x3_guide_bf16_fwd, + the following BatchNorm's
    statistics), so no fp32 output and no cast pass exist; the weight
    gradient from the bf16 gy and the bf16-rounded image on the MFMA kernel
    of stem.hip (mde_conv3x3_guide_bf16_wgrad; the image needs no gradient)."""

    @staticmethod
    def forward(ctx, x, weight, want_stats):
        x = x.contiguous()
        weight = weight.contiguous()
        n, _, h, w = x.shape
        cout = weight.shape[0]
        y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device)
        nb = _abi.query("mde_conv3x3_guide_bf16_stats_blocks", n, cout, h, w) if want_stats else 0
        stats = torch.empty((cout, nb, 4), dtype=torch.float32, device=x.device)
        _abi.call("mde_conv3x3_guide_bf16_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y),
                  _abi.ptr(stats) if nb else None, n, cout, h, w, _abi.stream_of(x))
        ctx.save_for_backward(x, weight)
        ctx.set_materialize_grads(False)  # no zero-fill launch for the extra output's gradient
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, gy, _gstats):
        if gy is None:  # only the non-differentiable output was used
            return (None, None, None)
        x, weight = ctx.saved_tensors
        gw = None
        if ctx.needs_input_grad[1]:
            n, cin, h, w = x.shape
            cout = weight.shape[0]
            gw = torch.empty_like(weight)
            if gy.dtype == torch.bfloat16 and w % 4 == 0:
                # bf16 gy read as such (stem.hip): no fp32 copy of the full-size gradient
                gy = gy.contiguous()
                ws = _ws(_abi.query("mde_conv3x3_guide_bf16_wgrad_workspace", n, cout, h, w), x)
                _abi.call("mde_conv3x3_guide_bf16_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw),
                          n, cout, h, w, _abi.ptr(ws), _abi.stream_of(gy))
            else:
                gyf = gy.float().contiguous()
                ws = _ws(_abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w,
                                    _abi.MDE_F32), x)
                _abi.call("mde_conv3x3_wgrad", _abi.ptr(gyf), _abi.ptr(x), _abi.ptr(gw), n, cin,
                          cout, h, w, _abi.ptr(ws), _abi.MDE_F32, _abi.stream_of(gyf))
        return None, gw, None


GUIDE_BF16 = os.environ.get("MDE_GUIDE_BF16", "1") != "0"  # A/B switch


def _conv3x3_apply(x, weight, passes, want_stats, gx_slot=None):
    if weight.dtype != torch.float32:
        raise TypeError(f"conv3x3: the HIP kernels take a float32 weight, got {weight.dtype}")
    cin, cout = x.shape[1], weight.shape[0]
    if (GUIDE_BF16 and cin == 3 and cout in (16, 32, 64) and passes[0] and x.dtype == torch.float32
            and _autocast_bf16(x) and not x.requires_grad
            and x.numel() < (1 << 31)):  # guide_ok's 32-bit image offsets (n*3*h*w)
        return _GuideConvBf16.apply(x, weight, bool(want_stats))
    if _conv3x3_bf16_path(cin, cout, x, weight):
        return _Conv3x3Bf16.apply(x.to(torch.bfloat16), weight, tuple(passes), want_stats)
    return _Conv3x3.apply(x, weight, tuple(passes), want_stats, gx_slot)


def conv3x3(x, weight, passes=(True, True, True), gx_slot=None):
    """Bias-free 3x3 / stride 1 / padding 1 convolution on the HIP MFMA kernel (per-pass flags)."""
    _gpu(x)
    return _conv3x3_apply(x, weight, passes, False, gx_slot)[0]


def conv3x3_stats(x, weight, passes=(True, True, True), gx_slot=None):
    """conv3x3 that also returns y's per-block BN statistics [cout][blocks][4]
    (shift, count, s1, s2) from the forward epilogue, or None when the forward
    is not on the HIP kernel (MIOpen)."""
    _gpu(x)
    y, stats = _conv3x3_apply(x, weight, passes, bool(passes[0]), gx_slot)
    return y, (stats if stats.shape[1] > 0 else None)


def conv_bn(conv: nn.Conv2d, bn: "BatchNorm2d", x, residual=None):
    """bn(conv(x)) with the conv bias folded into the BN kernel.

    Small-channel 1x1 convs run on the HIP MFMA pointwise kernel, small-channel
    3x3 convs on the HIP MFMA conv3x3 kernel (per pass, CONV3X3_HIP), the rest
    on MIOpen (PyTorch-ROCm)."""
    passes = conv3x3_passes(conv, x) if x.is_cuda else None
    want = bn.training or not bn.track_running_stats  # batch statistics: from the conv epilogue
    st = None
    if pointwise_ok(conv, x):
        _gpu(x)
        y = _Pointwise.apply(x, conv.weight)
    elif passes is not None:
        if want and passes[0] and _epilogue_stats_pay("conv3x3", conv, x):
            y, st = conv3x3_stats(x, conv.weight, passes)
        else:
            y = conv3x3(x, conv.weight, passes)
    elif stem_ok(conv, x):
        y = _StemBf16.apply(x, conv.weight)
    elif convbf_ok(conv, x):
        if want and _epilogue_stats_pay("convbf", conv, x):
            y, st = conv_bf16_stats(conv, x)
        else:
            y = conv_bf16(conv, x)
    elif conv3x3s2_ok(conv, x):
        y = _Conv3x3S2.apply(x, conv.weight)
    elif conv1x1_ok(conv, x):
        y = _Conv1x1.apply(x, conv.weight, conv.stride[0])
    else:
        y = torch.nn.functional.conv2d(x, conv.weight, None, conv.stride, conv.padding,
                                       conv.dilation, conv.groups)
    return batch_norm_act(y, bn, bn.act, residual, conv.bias, st)


_STATS_ROUTE: dict = {}


def _epilogue_stats_pay(kind, conv, x) -> bool:
    """Whether y's BN statistics from the conv epilogue save work: only when the
    BatchNorm's plane-mode apply merges the records itself (route 1 of
    mde_batchnorm_stats_route).  A separate merge launch costs about what the
    statistics pass it replaces does, and small tensors take the one-launch
    BatchNorm, which reads x once anyway."""
    n, cin, h, w = x.shape
    k, s = conv.kernel_size[0], conv.stride[0]
    key = (kind, n, cin, conv.out_channels, h, w, k, s, x.dtype)
    hit = _STATS_ROUTE.get(key)
    if hit is None:
        cout, pad = conv.out_channels, k // 2
        ho, wo = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
        if kind == "convbf":
            nb = _abi.query("mde_convbf_stats_blocks", n, cin, cout, h, w, k, s)
            dt = _abi.MDE_BF16
        else:
            dt = _abi.MDE_BF16 if (x.dtype == torch.bfloat16 or _autocast_bf16(x)) else _abi.MDE_F32
            nb = _abi.query("mde_conv3x3_stats_blocks", n, cin, cout, h, w, dt)
        hit = nb > 0 and _abi.query("mde_batchnorm_stats_route", n, cout, ho, wo, nb, dt) == 1
        _STATS_ROUTE[key] = hit
    return hit


def conv_nobias_stats(conv: nn.Conv2d, x, bn: nn.BatchNorm2d, gx_slot=None):
    """(conv_nobias(conv, x), statistics) where the statistics are y's per-block
    BN sums from the conv's epilogue when `bn` normalises with batch statistics,
    the conv runs on a HIP kernel that emits them (conv3x3 / convbf) and the
    BatchNorm consumes them without a merge launch (_epilogue_stats_pay), else
    None (the BatchNorm then takes its own statistics pass).  gx_slot: see
    residual_grad_slot (only for a conv that slot accepts)."""
    if x.is_cuda and (bn.training or not bn.track_running_stats):
        passes = conv3x3_passes(conv, x)
        if passes is not None:
            if passes[0] and _epilogue_stats_pay("conv3x3", conv, x):
                return conv3x3_stats(x, conv.weight, passes, gx_slot)
        elif convbf_ok(conv, x) and _epilogue_stats_pay("convbf", conv, x):
            return conv_bf16_stats(conv, x)
    return conv_nobias(conv, x, gx_slot), None


RESIDUAL_SLOT = os.environ.get("MDE_RES_SLOT", "1") != "0"  # A/B switch


def residual_grad_slot(conv: nn.Conv2d, x):
    """A GradSlot for a block input x that feeds both `conv` (a BasicBlock's
    first 3x3, DDRNet_23_slim.py:61-64) and the residual add of the block's
    last BatchNorm (:66-70), when conv's data gradient runs on the Winograd
    kernel in fp32: the BN backward puts the residual's gradient there and
    the Winograd data gradient adds it in its epilogue (mde_wino_conv_acc),
    so autograd's separate accumulation add (3 passes over x) disappears.
    None otherwise -- then nothing changes (a slot is only handed out where
    the conv is certain to take it: conv_nobias(_stats) routes such a conv to
    _Conv3x3)."""
    if not (RESIDUAL_SLOT and torch.is_grad_enabled() and x.is_cuda and x.requires_grad
            and x.dtype == torch.float32 and not _autocast_bf16(x)):
        return None
    passes = conv3x3_passes(conv, x)
    if passes is None or passes[1] != WINO:
        return None
    return GradSlot()


def conv_nobias(conv: nn.Conv2d, x, gx_slot=None):
    """conv(x) without its bias (folded into the following BN, or absent): the
    HIP 3x3 / stride-2 / 1x1 kernels where they apply (under bf16 autocast:
    the 16 / 32-channel bf16 3x3 kernels, then convbf.hip), else MIOpen."""
    passes = conv3x3_passes(conv, x) if x.is_cuda else None
    if passes is not None:
        return conv3x3(x, conv.weight, passes, gx_slot)
    if gx_slot is not None:
        raise RuntimeError("conv_nobias: a gradient slot for a conv off the HIP conv3x3 route")
    if convbf_ok(conv, x):
        return conv_bf16(conv, x)
    if conv3x3s2_ok(conv, x):
        return _Conv3x3S2.apply(x, conv.weight)
    if pointwise_ok(conv, x) and x.is_cuda and x.dtype == torch.float32 and not _autocast_bf16(x):
        return _Pointwise.apply(x, conv.weight)
    if conv1x1_ok(conv, x):
        return _Conv1x1.apply(x, conv.weight, conv.stride[0])
    if mm1x1_ok(conv, x):
        return conv1x1_mm(conv.weight, x)
    return torch.nn.functional.conv2d(x, conv.weight, None, conv.stride, conv.padding,
                                      conv.dilation, conv.groups)


def mm1x1_ok(conv: nn.Conv2d, x) -> bool:
    """A 1x1 / stride 1 / no padding conv under bf16 autocast that no HIP conv
    kernel takes (DAPPM's pooled branches, DDRNet_23_slim.py:121-160: 4x5,
    2x3, 1x2 and 1x1 planes with odd or tiny widths): a plain batched GEMM."""
    return (x.is_cuda and x.dim() == 4 and (_autocast_bf16(x) or x.dtype == torch.bfloat16)
            and conv.weight.dtype == torch.float32 and conv.kernel_size == (1, 1)
            and conv.stride == (1, 1) and conv.padding == (0, 0) and conv.dilation == (1, 1)
            and conv.groups == 1)


def conv1x1_mm(weight, x):
    """conv2d(x, weight) for a 1x1 kernel as y[n] = W . x[n] (rocBLAS batched
    GEMM on bf16 operands, fp32 accumulation: autocast's conv semantics) --
    NCHW in and out, none of MIOpen's NHWC transposes or zero fills."""
    n, cin, h, w = x.shape
    cout = weight.shape[0]
    wb = weight.view(cout, cin).to(torch.bfloat16)
    y = torch.matmul(wb, x.to(torch.bfloat16).reshape(n, cin, h * w))
    return y.view(n, cout, h, w)


CHANSUM = os.environ.get("MDE_CHANSUM", "1") != "0"  # A/B: 0 = autograd's bias-gradient sum


class _BiasAdd(torch.autograd.Function):
    """y + bias[None, :, None, None] (fp32 NCHW) whose bias gradient is
    mde_chansum (one fixed-order HBM-rate pass over gy) instead of autograd's
    grad.sum((0, 2, 3)) (~1.3 TB/s on the NewCRF projections' planes)."""

    @staticmethod
    def forward(ctx, y, bias):
        return y + bias.view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, gy):
        gb = None
        if ctx.needs_input_grad[1]:
            g = gy.contiguous()
            n, c, h, w = g.shape
            gb = torch.empty(c, dtype=torch.float32, device=g.device)
            ws = _ws(_abi.query("mde_chansum_workspace", n, c, h * w), g)
            _abi.call("mde_chansum", _abi.ptr(g), _abi.ptr(gb), n, c, h * w, _abi.ptr(ws), 0,
                      _abi.stream_of(g))
        return gy, gb


HEAD_CONV = os.environ.get("MDE_HEAD_CONV", "1") != "0"  # A/B: 0 = MIOpen


def head_conv_ok(conv: nn.Conv2d, x) -> bool:
    """A 3x3 / s1 / p1 conv with ONE output channel and a bias in fp32 (the
    NewCRF depth head, model_mobileV3_large_newCRFs.py Decoder.conv1) on
    head.hip's three VALU kernels."""
    return (HEAD_CONV and x.is_cuda and x.dtype == torch.float32 and not _autocast_bf16(x)
            and x.dim() == 4 and conv.out_channels == 1 and conv.bias is not None
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1
            and conv.weight.dtype == torch.float32
            and bool(_abi.query("mde_head_conv_supported", x.shape[0], x.shape[1], x.shape[2],
                                x.shape[3])))


class _HeadConv(torch.autograd.Function):
    """conv2d(x, W[1, C, 3, 3], b, padding=1) on head.hip: forward, data and
    weight gradients as HBM-rate VALU passes, the bias gradient by mde_chansum."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        x = x.contiguous()
        n, c, h, w = x.shape
        wt = weight.contiguous()
        y = torch.empty((n, 1, h, w), dtype=torch.float32, device=x.device)
        _abi.call("mde_head_conv_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(bias), _abi.ptr(y), n, c,
                  h, w, 0, _abi.stream_of(x))
        ctx.save_for_backward(x, wt)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wt = ctx.saved_tensors
        n, c, h, w = x.shape
        gy = gy.contiguous()
        st = _abi.stream_of(gy)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _abi.call("mde_head_conv_dgrad", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, c, h, w, 0,
                      st)
        if ctx.needs_input_grad[1]:
            gw = torch.empty_like(wt)
            ws = _ws(_abi.query("mde_head_conv_wgrad_workspace", n, c, h, w), gy)
            _abi.call("mde_head_conv_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, c, h, w,
                      _abi.ptr(ws), 0, st)
        if ctx.needs_input_grad[2]:
            gb = torch.empty(1, dtype=torch.float32, device=gy.device)
            ws = _ws(_abi.query("mde_chansum_workspace", n, 1, h * w), gy)
            _abi.call("mde_chansum", _abi.ptr(gy), _abi.ptr(gb), n, 1, h * w, _abi.ptr(ws), 0, st)
        return gx, gw, gb


class Conv2d(nn.Conv2d):
    """nn.Conv2d (same parameters and state_dict keys) whose bias-free
    forward takes conv_nobias's HIP kernels where they apply.  With a bias:
    a 3x3 / stride-1 conv with a HIP forward or data-gradient pass (the NewCRF
    projections, newcrf_layers.py: Winograd at 128-1024 channels), or a bf16
    autocast conv convbf.hip takes (DDRNet's segmenthead 1x1), runs on HIP and
    adds the bias in the output's dtype (its gradient is autograd's sum over
    the add); anything else -- and any padding_mode other than 'zeros' -- is
    the stock module (the DDRNet / decoder convs with a bias are folded into a
    BatchNorm by run_sequential / conv_bn instead)."""

    def forward(self, x):
        if x.is_cuda and self.padding_mode == "zeros":
            if self.bias is None:
                return conv_nobias(self, x)
            passes = conv3x3_passes(self, x)
            if passes is not None and (passes[0] or passes[1]):
                y = conv3x3(x, self.weight, passes)
                if CHANSUM and y.dtype == torch.float32 and _abi.query(
                        "mde_chansum_workspace", y.shape[0], y.shape[1], y.shape[2] * y.shape[3]):
                    return _BiasAdd.apply(y, self.bias)
                return y + self.bias.to(y.dtype).view(1, -1, 1, 1)
            if convbf_ok(self, x):
                y = conv_bf16(self, x)
                return y + self.bias.to(y.dtype).view(1, -1, 1, 1)
            if head_conv_ok(self, x):
                return _HeadConv.apply(x, self.weight, self.bias)
            if CHANSUM and conv1x1_ok(self, x):
                # a biased 1x1 (the NewCRF decoder's 960 -> 512 bridge,
                # model_mobileV3_large_newCRFs.py conv0) on the HIP 1x1 kernels
                y = _Conv1x1.apply(x, self.weight, self.stride[0])
                if _abi.query("mde_chansum_workspace", y.shape[0], y.shape[1],
                              y.shape[2] * y.shape[3]):
                    return _BiasAdd.apply(y, self.bias)
                return y + self.bias.view(1, -1, 1, 1)
        return super().forward(x)


def _bnrelu_pw_at(mods, i, x_shape) -> bool:
    """mods[i:i+5] = Conv(bias) -> BN(relu) -> ReLU slot -> Conv1x1(bias, HIP pointwise) -> BN."""
    if i + 4 >= len(mods):
        return False
    c0, b0, r0, c1, b1 = mods[i:i + 5]
    return (isinstance(c0, nn.Conv2d) and c0.bias is not None and c0.padding_mode == "zeros"
            and isinstance(b0, BatchNorm2d) and b0.act == "relu"
            and isinstance(r0, nn.Identity)
            and isinstance(c1, nn.Conv2d) and c1.bias is not None and isinstance(b1, BatchNorm2d)
            and c1.kernel_size == (1, 1) and c1.stride == (1, 1) and c1.padding == (0, 0)
            and c1.groups == 1 and c1.in_channels == c0.out_channels)


def run_sequential(seq: nn.Sequential, x):
    """Run a Sequential, folding every Conv2d(bias) -> BatchNorm2d pair (see conv_bn).

    Conv -> BN+ReLU -> 1x1 conv -> BN (the guided-upsampling branches,
    modules.py:43-74) additionally runs the first BN + ReLU inside the 1x1
    conv's operand load (bn_relu_pointwise) when the 1x1 conv is on HIP."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if x.is_cuda and _bnrelu_pw_at(mods, i, x.shape):
            # both BatchNorms take their statistics from the producing conv's
            # epilogue when that conv runs on a HIP kernel (train mode)
            want = mods[i + 1].training or not mods[i + 1].track_running_stats
            passes = conv3x3_passes(m, x)
            if passes is not None and want:
                y1, st1 = conv3x3_stats(x, m.weight, passes)
            else:
                y1, st1 = conv_nobias(m, x), None
            if pointwise_ok(mods[i + 3], y1):
                b2 = mods[i + 4]
                y2, st2 = bn_relu_pointwise(y1, mods[i + 1], m.bias, mods[i + 3], st1,
                                            b2.training or not b2.track_running_stats)
                x = batch_norm_act(y2, b2, b2.act, None, mods[i + 3].bias, st2)
                i += 5
                continue
            x = batch_norm_act(y1, mods[i + 1], mods[i + 1].act, None, m.bias, st1)
            i += 2
            continue
        if (isinstance(m, nn.Conv2d) and m.bias is not None and i + 1 < len(mods)
                and isinstance(mods[i + 1], BatchNorm2d) and m.padding_mode == "zeros"):
            x = conv_bn(m, mods[i + 1], x)
            i += 2
        elif (isinstance(m, Conv2d) and m.bias is None and i + 1 < len(mods)
              and isinstance(mods[i + 1], BatchNorm2d) and m.padding_mode == "zeros"):
            y, st = conv_nobias_stats(m, x, mods[i + 1])
            x = mods[i + 1](y, stats=st)
            i += 2
        else:
            x = m(x)
            i += 1
    return x


def run_sequential_raw(seq: nn.Sequential, x):
    """For Conv(bias) -> BN(relu) -> ReLU slot -> 1x1 Conv(bias) -> BN(relu) ->
    ReLU slot in training mode (fp32, or bf16 under autocast: the 3x3 conv on
    MIOpen bf16, the BN-ReLU-1x1 pair on its bf16 kernels): run it WITHOUT the last BatchNorm + ReLU
    and return (y2, stats2, bn2, conv2_bias) -- the last BN's raw input, its
    per-block statistics from the 1x1 conv's epilogue (None when that conv is
    not the HIP pointwise kernel), the BN module and its folded bias -- for a
    consumer that applies that BN itself (se_bn_cat, skip_reduce_bn).  None
    when the pattern or the conditions do not hold (then run_sequential)."""
    mods = list(seq)
    if (len(mods) != 6 or not x.is_cuda or x.dtype not in (torch.float32, torch.bfloat16)
            or not _bnrelu_pw_at(mods, 0, x.shape)
            or not isinstance(mods[5], nn.Identity) or mods[4].act != "relu"
            or not mods[1].training or not mods[4].training):
        return None
    m, c1 = mods[0], mods[3]
    k = m.kernel_size
    same = (m.stride == (1, 1) and m.dilation == (1, 1) and k[0] % 2 == 1 and k[1] % 2 == 1
            and m.padding == (k[0] // 2, k[1] // 2))
    passes = conv3x3_passes(m, x)
    if passes is not None:
        y1, st1 = conv3x3_stats(x, m.weight, passes)
    else:
        y1, st1 = conv_nobias(m, x), None
    if same and pointwise_ok(c1, x):  # y1 keeps x's H x W, which pointwise_ok checked
        y2, st2 = bn_relu_pointwise(y1, mods[1], m.bias, c1, st1, True)
        return y2, st2, mods[4], c1.bias
    x1 = batch_norm_act(y1, mods[1], "relu", None, m.bias, st1)
    y2 = torch.nn.functional.conv2d(x1, c1.weight, None, c1.stride, c1.padding, c1.dilation,
                                    c1.groups)
    return y2, None, mods[4], c1.bias


class _SkipReduceBN(torch.autograd.Function):
    """reduce(relu(bn(r + prebias)) + d) (the comb_conv's last BatchNorm + ReLU
    and the skip fusion, modules.py:72-73,100) with the BN + ReLU applied in
    the skip kernel's operand load: the BN output is never written, and the
    skip backward forms the BN backward's sums where the shape allows, so the
    BN runs its apply pass only."""

    @staticmethod
    @_bn_fwd
    def forward(ctx, r, d, weight, bias, gamma, beta, prebias, meta, stats, d_slot=None):
        # bf16 storage when r is bf16 (autocast), else fp32; d follows r
        dt = torch.bfloat16 if r.dtype == torch.bfloat16 else torch.float32
        r, d = r.to(dt).contiguous(), d.to(dt).contiguous()
        n, cin, h, w = r.shape
        cout = weight.shape[0]
        wm = weight.reshape(cout, cin).contiguous()
        f32 = dict(dtype=torch.float32, device=r.device)
        scale, shift = torch.empty(cin, **f32), torch.empty(cin, **f32)
        mean, invstd = torch.empty(cin, **f32), torch.empty(cin, **f32)
        rm, rv, nbt, momentum, eps = meta
        st = _abi.stream_of(r)
        ws = _ws(_abi.query("mde_batchnorm_workspace", n, cin, h, w), r)
        if stats is not None:
            _abi.call("mde_batchnorm_fwd_coef_stats", _abi.ptr(r), _abi.ptr(gamma), _abi.ptr(beta),
                      _abi.ptr(prebias), _abi.ptr(rm), _abi.ptr(rv), _abi.ptr(nbt), float(momentum),
                      float(eps), _abi.ptr(scale), _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(invstd),
                      n, cin, h, w, _abi.ptr(stats), stats.shape[1], _abi.ptr(ws),
                      _abi.dtype_code(r), st)
        else:
            _abi.call("mde_batchnorm_fwd_coef", _abi.ptr(r), _abi.ptr(gamma), _abi.ptr(beta),
                      _abi.ptr(prebias), _abi.ptr(rm), _abi.ptr(rv), _abi.ptr(nbt), float(momentum),
                      float(eps), 1, _abi.ptr(scale), _abi.ptr(shift), _abi.ptr(mean),
                      _abi.ptr(invstd), n, cin, h, w, _abi.ptr(ws), _abi.dtype_code(r), st)
        out = torch.empty((n, cout, h, w), dtype=dt, device=r.device)
        _abi.call("mde_skip_reduce_bn_fwd", _abi.ptr(r), _abi.ptr(d), _abi.ptr(scale),
                  _abi.ptr(shift), _abi.ptr(wm), _abi.ptr(bias), _abi.ptr(out), n, cin, cout, h, w,
                  _abi.dtype_code(r), st)
        ctx.save_for_backward(r, d, wm, gamma, beta, scale, shift, mean, invstd)
        ctx.wshape, ctx.has_pb, ctx.d_slot = weight.shape, prebias is not None, d_slot
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, gout):
        r, d, wm, gamma, beta, scale, shift, mean, invstd = ctx.saved_tensors
        gout = gout.to(r.dtype).contiguous()
        n, cin, h, w = r.shape
        cout = wm.shape[0]
        st = _abi.stream_of(gout)
        gs = torch.empty_like(r)  # d/d(relu output) == d/dd
        gw, gb = torch.empty_like(wm), torch.empty(cout, dtype=torch.float32, device=r.device)
        use_sums = bool(_abi.query("mde_skip_reduce_bn_supported", cin, cout, h, w, 1))
        sums = torch.empty((cin, 2), dtype=torch.float32, device=r.device) if use_sums else None
        ws = _ws(_abi.query("mde_skip_reduce_bn_workspace", n, cin, cout, h, w), r)
        _abi.call("mde_skip_reduce_bn_bwd", _abi.ptr(gout), _abi.ptr(r), _abi.ptr(d),
                  _abi.ptr(scale), _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(wm), _abi.ptr(gs),
                  _abi.ptr(gw), _abi.ptr(gb), _abi.ptr(sums), n, cin, cout, h, w, _abi.ptr(ws),
                  _abi.dtype_code(gout), st)
        gr = torch.empty_like(r)
        gg, gbeta = torch.empty_like(gamma), torch.empty_like(beta)
        gpb = torch.empty_like(gamma) if (ctx.has_pb and ctx.needs_input_grad[6]) else None
        if sums is not None:
            _abi.call("mde_batchnorm_bwd_apply", _abi.ptr(gs), _abi.ptr(r), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(sums),
                      _abi.ptr(gr), None, _abi.ptr(gg), _abi.ptr(gbeta), _abi.ptr(gpb), n, cin, h,
                      w, _ACTS["relu"], _abi.dtype_code(gout), st)
        else:
            ws2 = _ws(_abi.query("mde_batchnorm_workspace", n, cin, h, w), r)
            _abi.call("mde_batchnorm_bwd", _abi.ptr(gs), _abi.ptr(r), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(gr), None,
                      _abi.ptr(gg), _abi.ptr(gbeta), _abi.ptr(gpb), n, cin, h, w, _ACTS["relu"],
                      _abi.ptr(ws2), _abi.dtype_code(gout), st)
        if ctx.d_slot is not None and ctx.needs_input_grad[1]:
            ctx.d_slot.put(gs)  # d's producer sums it on load (functional.GradSlot)
            gd = None
        else:
            gd = gs
        return gr, gd, gw.view(ctx.wshape), gb, gg, gbeta, gpb, None, None, None


def skip_reduce_bn_ok(r, cout: int) -> bool:
    """Whether skip_reduce_bn has a kernel for this (raw input, output channels)."""
    return (r.dim() == 4 and r.dtype in (torch.float32, torch.bfloat16) and
            bool(_abi.query("mde_skip_reduce_bn_supported", r.shape[1], cout, r.shape[2],
                            r.shape[3], 0)))


def skip_reduce_bn(r, bn: nn.BatchNorm2d, prebias, d, weight, bias, stats=None):
    """reduce(relu(bn(r + prebias)) + d) (modules.py:72-73,100) on the fused HIP
    path: r is the comb_conv's last 1x1 conv output without its bias (folded
    as `prebias`), bn its training-mode BatchNorm, stats r's per-block
    statistics from that conv's epilogue (or None: a statistics pass).  When
    d carries a GradSlot (functional.bilinear_resize_x2_slotted) d's gradient
    goes there instead of through autograd."""
    _gpu(r, d, prebias, weight, bias)
    if bn.weight is None or bn.bias is None or bn.momentum is None or not bn.training:
        raise NotImplementedError("skip_reduce_bn needs an affine, momentum, training-mode BatchNorm")
    track = bn.track_running_stats
    meta = (bn.running_mean if track else None, bn.running_var if track else None,
            bn.num_batches_tracked if track else None, bn.momentum, bn.eps)
    return _SkipReduceBN.apply(r, d, weight, bias, bn.weight, bn.bias, prebias, meta, stats,
                               getattr(d, "_mde_grad_slot", None))


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d on HIP kernels with an optional fused activation."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, act="none", **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        if act not in _ACTS:
            raise ValueError(f"act must be one of {sorted(_ACTS)}")
        self.act = act

    def forward(self, x, residual=None, prebias=None, stats=None, act=None, res_slot=None):
        """act overrides the module's activation for this call (a caller that
        applies the reference's following ReLU in this pass, e.g. DualResNet's
        `self.relu(x)` of an output nothing else reads); res_slot: see
        batch_norm_act."""
        return batch_norm_act(x, self, self.act if act is None else act, residual, prebias, stats,
                              res_slot)

    def extra_repr(self):
        return super().extra_repr() + f", act={self.act}"


class _DWConv(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, x, weight, k, stride, pad):
        x = x.contiguous()
        n, c, h, w = x.shape
        ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
        y = torch.empty((n, c, ho, wo), dtype=x.dtype, device=x.device)
        _abi.call("mde_dwconv_fwd", _abi.ptr(x), _abi.ptr(weight), _abi.ptr(y), n, c, h, w, k,
                  stride, pad, _abi.dtype_code(x), _abi.stream_of(x))
        ctx.save_for_backward(x, weight)
        ctx.meta = (k, stride, pad)
        return y

    @staticmethod
    @_amp_bwd
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        k, stride, pad = ctx.meta
        gy = gy.contiguous()
        n, c, h, w = x.shape
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw = torch.empty_like(weight) if ctx.needs_input_grad[1] else None
        ws = _ws(_abi.query("mde_dwconv_workspace", n, c, h, w, k, stride, pad), x) \
            if gw is not None else None
        if gx is not None or gw is not None:
            _abi.call("mde_dwconv_bwd", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(weight), _abi.ptr(gx),
                      _abi.ptr(gw), n, c, h, w, k, stride, pad, _abi.ptr(ws),
                      _abi.dtype_code(gy), _abi.stream_of(gy))
        return gx, gw, None, None, None


def depthwise_conv2d(x, conv: nn.Conv2d):
    """Depthwise nn.Conv2d (groups == in == out, square k3/k5, stride 1/2) on the HIP kernel."""
    _gpu(x)
    k = conv.kernel_size[0]
    s = conv.stride[0]
    p = conv.padding[0]
    if (conv.kernel_size != (k, k) or k not in (3, 5) or conv.stride != (s, s) or s not in (1, 2)
            or conv.padding != (p, p) or conv.dilation != (1, 1) or conv.padding_mode != "zeros"
            or not (conv.groups == conv.in_channels == conv.out_channels)):
        raise NotImplementedError(f"no HIP depthwise kernel for {conv}")
    y = _DWConv.apply(x, conv.weight, k, s, p)
    if conv.bias is not None:
        y = y + conv.bias.view(1, -1, 1, 1)
    return y


def depthwise_conv_bn_act(x, conv: nn.Conv2d, bn: "BatchNorm2d", act: str = "none"):
    """act(bn(depthwise_conv(x))) — MobileNetV3's k3/k5 depthwise stage, both on HIP kernels."""
    return batch_norm_act(depthwise_conv2d(x, conv), bn, act)


class _SEGate(torch.autograd.Function):
    @staticmethod
    @_amp_fwd
    def forward(ctx, x, w1, b1, w2, b2):
        x = x.contiguous()
        n, c, h, w = x.shape
        cr = w1.shape[0]
        ctx.wshapes = (w1.shape, w2.shape)
        w1 = w1.reshape(cr, c).contiguous()
        w2 = w2.reshape(c, cr).contiguous()
        out = torch.empty_like(x)
        s = torch.empty((n, c), dtype=torch.float32, device=x.device)
        hidden = torch.empty((n, cr), dtype=torch.float32, device=x.device)
        mean = torch.empty((n, c), dtype=torch.float32, device=x.device)
        ws = _ws(_abi.query("mde_se_workspace", n, c, cr, h, w), x)
        _abi.call("mde_se_gate_fwd", _abi.ptr(x), c, None, 0, _abi.ptr(w1), _abi.ptr(b1),
                  _abi.ptr(w2), _abi.ptr(b2), cr, 1, _abi.ptr(out), _abi.ptr(s), _abi.ptr(hidden),
                  _abi.ptr(mean), n, h, w, _abi.ptr(ws), _abi.dtype_code(x), _abi.stream_of(x))
        ctx.save_for_backward(x, w1, w2, b2, s, hidden, mean)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, gout):
        x, w1, w2, b2, s, hidden, mean = ctx.saved_tensors
        gout = gout.contiguous()
        n, c, h, w = x.shape
        cr = w1.shape[0]
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
        gb1 = torch.empty(cr, dtype=x.dtype, device=x.device)
        gb2 = torch.empty(c, dtype=x.dtype, device=x.device)
        ws = _ws(_abi.query("mde_se_workspace", n, c, cr, h, w), x)
        _abi.call("mde_se_gate_bwd", _abi.ptr(gout), _abi.ptr(x), c, None, 0, _abi.ptr(w1),
                  _abi.ptr(w2), _abi.ptr(b2), cr, 1, _abi.ptr(s), _abi.ptr(hidden),
                  _abi.ptr(mean), _abi.ptr(gx), None, _abi.ptr(gw1), _abi.ptr(gb1), _abi.ptr(gw2),
                  _abi.ptr(gb2), n, h, w, _abi.ptr(ws), _abi.dtype_code(gout),
                  _abi.stream_of(gout))
        return gx, gw1.view(ctx.wshapes[0]), gb1, gw2.view(ctx.wshapes[1]), gb2


def se_hardsigmoid(x, fc1: nn.Conv2d, fc2: nn.Conv2d):
    """x * hardsigmoid(fc2(relu(fc1(avgpool(x))))) (torchvision.ops.SqueezeExcitation) on HIP.

    fc1 / fc2 are the 1x1 convolutions with bias of the reference module; the
    squeeze, both FCs, the gate and the rescale run in mde_se_gate_{fwd,bwd}.
    """
    _gpu(x)
    if fc1.bias is None or fc2.bias is None:
        raise NotImplementedError("torchvision SqueezeExcitation has fc biases")
    return _SEGate.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
