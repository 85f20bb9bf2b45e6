"""GPU parity of the HIP MFMA 3x3 convolution (mde_conv3x3_*) against the CPU oracle.

The reference layer is `nn.Conv2d(c_in, E, kernel_size=3, padding=1)` of the
guided-upsampling blocks (src/GuideDepth/model/modules.py:43-74); its CPU
arithmetic (ATen conv2d, the reference's own dependency) evaluated in float64
is the oracle.  Tolerance: 1e-5 of the output's max magnitude for the forward
and data gradient (fp32 sums of 27-288 products), 2e-5 for the weight
gradient (fp32 sums over up to 10^7 pixels, reduced in a fixed order).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
PAIRS = [(3, 16), (3, 32), (3, 64), (16, 16), (32, 32)]
# (n, h, w): tile-aligned, ragged rows/cols, w % 4 != 0, a single pixel,
# w % 4 == 0 with a partial column tile (the guide convs' staged stores)
SIZES = [(2, 16, 64), (1, 13, 70), (2, 9, 37), (1, 1, 1), (3, 20, 130), (2, 11, 100)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    import monocular_depth_estimation_amd  # noqa: F401


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _case(cin, cout, n, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), generator=g) - 0.5) * 0.3
    gy = torch.rand((n, cout, h, w), generator=g) - 0.5
    return x, wt, gy


@pytest.mark.parametrize("cin,cout", PAIRS)
@pytest.mark.parametrize("n,h,w", SIZES)
def test_conv3x3_vs_float64_oracle(cin, cout, n, h, w):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import conv3x3
    x, wt, gy = _case(cin, cout, n, h, w, 100 * cin + cout + h)
    xr = x.double().requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, 1)
    yr.backward(gy.double())
    passes = tuple(bool(_abi.query("mde_conv3x3_supported", cin, cout, i, 0)) for i in range(3))
    assert passes[0] and passes[2]
    xg = x.to(DEV).requires_grad_(passes[1])
    wg = wt.to(DEV).requires_grad_(True)
    y = conv3x3(xg, wg, passes)
    y.backward(gy.to(DEV))
    assert rel_err(y, yr) <= 1e-5, "forward"
    assert rel_err(wg.grad, wr.grad) <= 2e-5, "weight gradient"
    if passes[1]:
        assert rel_err(xg.grad, xr.grad) <= 1e-5, "data gradient"


@pytest.mark.parametrize("cin,cout,h,w", [(16, 16, 480, 640), (3, 16, 480, 640), (32, 32, 240, 320),
                                          (3, 64, 120, 160)])
def test_conv3x3_full_size_vs_miopen(cin, cout, h, w):
    """BASELINE cfg2 shapes (bs 4 of 32): HIP vs MIOpen fp32, all three passes."""
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import conv3x3
    gen = torch.Generator(device=DEV).manual_seed(cin * cout)
    x = torch.rand((4, cin, h, w), device=DEV, generator=gen) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), device=DEV, generator=gen) - 0.5) * 0.3
    gy = torch.rand((4, cout, h, w), device=DEV, generator=gen) - 0.5
    passes = tuple(bool(_abi.query("mde_conv3x3_supported", cin, cout, i, 0)) for i in range(3))
    xh = x.clone().requires_grad_(passes[1])
    wh = wt.clone().requires_grad_(True)
    y = conv3x3(xh, wh, passes)
    y.backward(gy)
    xm = x.clone().requires_grad_(True)
    wm = wt.clone().requires_grad_(True)
    ym = torch.nn.functional.conv2d(xm, wm, None, 1, 1)
    ym.backward(gy)
    assert rel_err(y, ym) <= 2e-5
    assert rel_err(wh.grad, wm.grad) <= 1e-4
    if passes[1]:
        assert rel_err(xh.grad, xm.grad) <= 2e-5


# Wide channels (DDRNet 64/128/256): weight gradient only; (n, h, w) cover
# the fixed-strip kernel at the cfg2 widths (80-column strips of one row, 40 /
# 20 whole rows), 80-column strips side by side (160, 240: halo columns from
# the neighbouring strip), a ragged last row tile, w > 126 off the strip
# widths (generic 64-column strips with a ragged last strip), one row, and
# non-square channel pairs.
WIDE = [(64, 64, 2, 60, 80), (128, 128, 2, 30, 40), (256, 256, 2, 15, 20),
        (64, 64, 1, 9, 160), (128, 64, 1, 5, 240), (64, 64, 1, 7, 130), (64, 64, 3, 1, 5),
        (32, 128, 1, 9, 21), (64, 64, 1, 33, 200)]


# 32 -> 32 at widths that are multiples of 80: the fixed-strip kernel with
# 32-channel output groups (DDRNet layer1 at 120x160, decoder at 240x320)
@pytest.mark.parametrize("n,h,w", [(2, 30, 160), (1, 7, 80), (2, 5, 320)])
def test_conv3x3_wgrad_c32_strips_vs_float64(n, h, w):
    from monocular_depth_estimation_amd.nn import conv3x3
    x, wt, gy = _case(32, 32, n, h, w, 11 + h)
    wr = wt.double().requires_grad_(True)
    torch.nn.functional.conv2d(x.double(), wr, None, 1, 1).backward(gy.double())
    wg = wt.to(DEV).requires_grad_(True)
    conv3x3(x.to(DEV), wg, (False, False, True)).backward(gy.to(DEV))
    assert rel_err(wg.grad, wr.grad) <= 2e-5


@pytest.mark.parametrize("cin,cout,n,h,w", WIDE)
def test_conv3x3_wide_wgrad_vs_float64_oracle(cin, cout, n, h, w):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import conv3x3
    x, wt, gy = _case(cin, cout, n, h, w, 7 * cin + cout + h)
    xr = x.double()
    wr = wt.double().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, None, 1, 1).backward(gy.double())
    passes = tuple(bool(_abi.query("mde_conv3x3_supported", cin, cout, i, 0)) for i in range(3))
    assert passes == (False, False, True)
    wg = wt.to(DEV).requires_grad_(True)
    conv3x3(x.to(DEV), wg, passes).backward(gy.to(DEV))
    assert rel_err(wg.grad, wr.grad) <= 2e-5


# padded input channels (round 6): the NewCRF projections' 24 / 40 / 112 ->
# 128 / 256 / 512 (newcrf_layers.py:384-392) on the fixed-strip widths, ragged
# row counts; other widths are not taken (workspace 0)
@pytest.mark.parametrize("cin,cout,n,h,w", [(24, 128, 2, 33, 160), (40, 256, 2, 17, 80),
                                            (112, 512, 3, 30, 40), (56, 64, 2, 9, 20)])
def test_conv3x3_wide_wgrad_padded_channels_vs_float64(cin, cout, n, h, w):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import conv3x3
    assert _abi.query("mde_conv3x3_supported", cin, cout, 2, 0)
    assert _abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w, 0) > 0
    assert _abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, 48, 0) == 0
    x, wt, gy = _case(cin, cout, n, h, w, 5 * cin + cout + h)
    wr = wt.double().requires_grad_(True)
    torch.nn.functional.conv2d(x.double(), wr, None, 1, 1).backward(gy.double())
    wg = wt.to(DEV).requires_grad_(True)
    conv3x3(x.to(DEV), wg, (False, False, True)).backward(gy.to(DEV))
    assert rel_err(wg.grad, wr.grad) <= 2e-5


def test_conv3x3_wide_wgrad_deterministic():
    from monocular_depth_estimation_amd.nn import conv3x3
    x, wt, gy = _case(128, 128, 4, 30, 40, 9)
    outs = []
    for _ in range(2):
        wg = wt.to(DEV).requires_grad_(True)
        conv3x3(x.to(DEV), wg, (False, False, True)).backward(gy.to(DEV))
        outs.append(wg.grad.cpu())
    assert torch.equal(outs[0], outs[1])


def test_conv3x3_deterministic():
    from monocular_depth_estimation_amd.nn import conv3x3
    x, wt, gy = _case(16, 16, 2, 50, 90, 3)
    outs = []
    for _ in range(2):
        xg = x.to(DEV).requires_grad_(True)
        wg = wt.to(DEV).requires_grad_(True)
        y = conv3x3(xg, wg)
        y.backward(gy.to(DEV))
        outs.append((y.detach().cpu(), xg.grad.cpu(), wg.grad.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_conv3x3_unsupported_shape_raises():
    from monocular_depth_estimation_amd import _abi
    x = torch.rand((1, 8, 4, 4), device=DEV)
    w = torch.rand((8, 8, 3, 3), device=DEV)
    y = torch.empty((1, 8, 4, 4), device=DEV)
    assert not _abi.query("mde_conv3x3_supported", 8, 8, 0, 0)
    with pytest.raises(_abi.MdeError, match="unsupported"):
        _abi.call("mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(w), _abi.ptr(y), 1, 8, 8, 4, 4, 0,
                  _abi.stream_of(x))


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("cin,e,eo,h,w", [(16, 16, 8, 32, 64), (3, 32, 16, 16, 48), (64, 64, 32, 8, 64),
                                           (64, 64, 64, 8, 64)])
def test_fused_bn_relu_pointwise_branch_vs_float64(cin, e, eo, h, w, train):
    """conv3x3 -> BN+ReLU -> 1x1 -> BN+ReLU (a guided-upsampling branch,
    modules.py:43-49) on the fused HIP path (BN1+ReLU inside the 1x1 conv's
    operand load) vs the same Sequential as plain torch modules in float64:
    output, input gradient, every parameter gradient and the BN running stats.
    e -> eo = 64 -> 64 is up_1's comb_conv (GuideDepth.py:21-33)."""
    import copy

    from monocular_depth_estimation_amd.GuideDepth.model.modules import _conv_bn_relu
    from monocular_depth_estimation_amd.nn import BatchNorm2d, run_sequential
    torch.manual_seed(cin + e + h)
    seq = torch.nn.Sequential(*_conv_bn_relu(cin, e, 3), *_conv_bn_relu(e, eo, 1))
    for m in seq.modules():
        if isinstance(m, BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 2.0)
    ref = torch.nn.Sequential(*[torch.nn.BatchNorm2d(m.num_features) if isinstance(m, BatchNorm2d)
                                else (torch.nn.ReLU() if isinstance(m, torch.nn.Identity) else
                                      copy.deepcopy(m)) for m in seq]).double()
    for r, m in zip(ref, seq):
        if isinstance(m, BatchNorm2d):
            r.load_state_dict(m.state_dict())
    ref.train(train)
    seq = seq.to(DEV).train(train)
    x = torch.rand((2, cin, h, w)) - 0.5
    gy = torch.rand((2, eo, h, w)) - 0.5
    xg = x.to(DEV).requires_grad_(True)
    y = run_sequential(seq, xg)
    y.backward(gy.to(DEV))
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy.double())
    assert rel_err(y, yr) <= 1e-4
    assert rel_err(xg.grad, xr.grad) <= 1e-3
    for (n1, p1), (n2, p2) in zip(seq.named_parameters(), ref.named_parameters()):
        # a conv bias in front of a train-mode BN has an identically zero
        # gradient (the batch mean absorbs it): compare on an absolute floor
        err = float((p1.grad.double().cpu() - p2.grad).abs().max())
        assert err <= 1e-3 * max(float(p2.grad.abs().max()), 1e-6), n1
    for b1, b2 in zip(seq.buffers(), ref.buffers()):
        assert rel_err(b1, b2) <= 1e-5


@pytest.mark.parametrize("cin,cout,n,h,w", [(16, 8, 8, 96, 128), (32, 32, 4, 60, 80), (32, 16, 3, 8, 64),
                                             (16, 32, 2, 16, 64)])
def test_pointwise_bwd_bn_sums_match_separate_reduce(cin, cout, n, h, w):
    """mde_pointwise_bwd_bn's epilogue sums + mde_batchnorm_bwd_apply == the
    unfused mde_pointwise_bwd + mde_batchnorm_bwd (its own reduce pass): same
    gx of the 1x1 conv bit for bit, BN input / parameter gradients to 1e-5."""
    from monocular_depth_estimation_amd import _abi
    g = torch.Generator().manual_seed(cin * cout + h)
    f = dict(device=DEV, dtype=torch.float32)
    y1 = (torch.rand((n, cin, h, w), generator=g) * 2 - 0.7).to(DEV)
    gy2 = (torch.rand((n, cout, h, w), generator=g) - 0.5).to(DEV)
    w2 = (torch.rand((cout, cin), generator=g) - 0.5).to(DEV)
    gamma = (torch.rand(cin, generator=g) + 0.5).to(DEV)
    beta = (torch.rand(cin, generator=g) - 0.5).to(DEV)
    mean = y1.mean(dim=(0, 2, 3))
    invstd = 1.0 / torch.sqrt(y1.var(dim=(0, 2, 3), unbiased=False) + 1e-5)
    scale = gamma * invstd
    shift = beta - mean * scale
    st = _abi.stream_of(y1)
    ws = torch.empty(_abi.query("mde_pointwise_workspace", n, cin, cout, h, w) // 4 + 1, **f)
    outs = []
    for fused in (False, True):
        gz, gw2 = torch.empty_like(y1), torch.empty_like(w2)
        gy1, gg, gb = torch.empty_like(y1), torch.empty(cin, **f), torch.empty(cin, **f)
        if fused:
            sums = torch.empty((cin, 2), **f)
            _abi.call("mde_pointwise_bwd_bn", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(w2), _abi.ptr(gz), _abi.ptr(gw2),
                      _abi.ptr(sums), n, cin, cout, h, w, _abi.ptr(ws), 0, st)
            _abi.call("mde_batchnorm_bwd_apply", _abi.ptr(gz), _abi.ptr(y1), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(sums),
                      _abi.ptr(gy1), None, _abi.ptr(gg), _abi.ptr(gb), None, n, cin, h, w, 1, 0, st)
        else:
            _abi.call("mde_pointwise_bwd", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(w2), _abi.ptr(gz), _abi.ptr(gw2), n, cin, cout, h,
                      w, _abi.ptr(ws), 0, st)
            ws2 = torch.empty(_abi.query("mde_batchnorm_workspace", n, cin, h, w) // 4 + 1, **f)
            _abi.call("mde_batchnorm_bwd", _abi.ptr(gz), _abi.ptr(y1), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(gy1), None,
                      _abi.ptr(gg), _abi.ptr(gb), None, n, cin, h, w, 1, _abi.ptr(ws2), 0, st)
        outs.append((gz, gw2, gy1, gg, gb))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    for a, b, what in zip(outs[1][2:], outs[0][2:], ("gy1", "ggamma", "gbeta")):
        assert rel_err(a, b) <= 1e-5, what


def test_pointwise_bwd_bn_cin64_unsupported():
    from monocular_depth_estimation_amd import _abi
    f = dict(device=DEV, dtype=torch.float32)
    n, cin, cout, h, w = 1, 64, 32, 8, 8
    x, gy = torch.rand((n, cin, h, w), **f), torch.rand((n, cout, h, w), **f)
    v = torch.rand(cin, **f)
    ws = torch.empty(_abi.query("mde_pointwise_workspace", n, cin, cout, h, w) // 4 + 1, **f)
    with pytest.raises(_abi.MdeError, match="unsupported"):
        _abi.call("mde_pointwise_bwd_bn", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(v), _abi.ptr(v),
                  _abi.ptr(v), _abi.ptr(torch.rand((cout, cin), **f)), _abi.ptr(torch.empty_like(x)),
                  _abi.ptr(torch.empty((cout, cin), **f)), _abi.ptr(torch.empty((cin, 2), **f)), n,
                  cin, cout, h, w, _abi.ptr(ws), 0, _abi.stream_of(x))



@pytest.mark.parametrize("cin,cout,n,h,w,off", [(16, 16, 4, 120, 160, 0.0), (3, 32, 3, 37, 70, 0.0),
                                                (16, 16, 2, 30, 64, 100.0), (3, 64, 2, 16, 48, 5.0)])
def test_bn_statistics_from_conv_epilogue(cin, cout, n, h, w, off):
    """BatchNorm (train) fed the conv3x3 forward epilogue's per-block shifted
    sums == the same BatchNorm with its own statistics pass: output,
    running mean / var, saved statistics (through the backward) -- also when
    |mean| >> std (input offset)."""
    import copy

    from monocular_depth_estimation_amd.nn import BatchNorm2d, batch_norm_act, conv3x3_stats
    g = torch.Generator().manual_seed(cin + cout + h)
    x = (torch.rand((n, cin, h, w), generator=g) - 0.5 + off).to(DEV)
    wt = ((torch.rand((cout, cin, 3, 3), generator=g) - 0.5) * 0.3).to(DEV)
    y, st = conv3x3_stats(x, wt)
    assert st is not None and st.shape[0] == cout
    assert float(st[:, :, 1].sum()) == n * h * w * cout  # every output counted once
    bn = BatchNorm2d(cout, act="relu").to(DEV).train()
    bn2 = copy.deepcopy(bn)
    ya = batch_norm_act(y.detach().requires_grad_(True), bn, "relu", None, None, st)
    yb = batch_norm_act(y.detach().requires_grad_(True), bn2, "relu")
    # both fp32 paths against float64 batch statistics of the same y: the
    # epilogue statistics may not be worse than the statistics pass (2x +
    # floor; with |mean| >> std both carry the mean's fp32 rounding)
    y64 = y.double()
    m64 = y64.mean(dim=(0, 2, 3), keepdim=True)
    v64 = y64.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    ref = torch.relu((y64 - m64) / torch.sqrt(v64 + bn.eps) * bn.weight.double().view(1, -1, 1, 1)
                     + bn.bias.double().view(1, -1, 1, 1))
    ea, eb = rel_err(ya, ref), rel_err(yb, ref)
    assert ea <= max(2.0 * eb, 1e-6), (ea, eb)
    scale = float((y64 - m64).abs().max())  # means ~0 here: compare on y's centred scale
    assert float((bn.running_mean - bn2.running_mean).abs().max()) <= 1e-6 * max(scale, 1.0)
    assert rel_err(bn.running_var, bn2.running_var) <= 2e-5


# (64, 64): two 64 -> 32 launches writing channel halves + their statistics rows
@pytest.mark.parametrize("cin,cout,n,h,w", [(16, 8, 4, 96, 128), (64, 32, 2, 60, 80), (32, 16, 3, 8, 64),
                                            (64, 64, 2, 60, 80)])
def test_bn_statistics_from_pointwise_epilogue(cin, cout, n, h, w):
    """The BN-ReLU-fed 1x1 conv's forward epilogue statistics for the next
    BatchNorm == that BatchNorm's own statistics pass."""
    import copy

    from monocular_depth_estimation_amd.nn import BatchNorm2d, batch_norm_act, bn_relu_pointwise
    g = torch.Generator().manual_seed(cin * cout + h)
    y1 = (torch.rand((n, cin, h, w), generator=g) * 2 - 0.7).to(DEV)
    bn1 = BatchNorm2d(cin, act="relu").to(DEV).train()
    conv = torch.nn.Conv2d(cin, cout, 1).to(DEV)
    y2, st2 = bn_relu_pointwise(y1, bn1, None, conv, None, True)
    assert st2 is not None and float(st2[:, :, 1].sum()) == n * h * w * cout
    bn2 = BatchNorm2d(cout, act="relu").to(DEV).train()
    bn3 = copy.deepcopy(bn2)
    za = batch_norm_act(y2.detach(), bn2, "relu", None, None, st2)
    zb = batch_norm_act(y2.detach(), bn3, "relu")
    assert rel_err(za, zb) <= 2e-6
    assert rel_err(bn2.running_var, bn3.running_var) <= 2e-5


# ----------------------------------------------------------------- bf16 (cfg3)
BF_PAIRS = [(16, 16), (32, 32)]
# w % 4 == 0 (the bf16 kernels' 8-byte column chunks); ragged tiles and rows
BF_SIZES = [(2, 16, 64), (1, 13, 72), (3, 20, 132), (1, 1, 4), (2, 37, 200)]


def _bf(t):
    return t.to(torch.bfloat16).double()


@pytest.mark.parametrize("cin,cout", BF_PAIRS)
@pytest.mark.parametrize("n,h,w", BF_SIZES)
def test_conv3x3_bf16_vs_float64_oracle(cin, cout, n, h, w):
    """The v_mfma_f32_16x16x32_bf16 kernels (autocast's conv semantics: bf16
    x / gy, the fp32 weight rounded to bf16, fp32 accumulation, bf16 y / gx,
    fp32 weight gradient) against float64 convolutions of the SAME rounded
    operands.  y and gx are the exact sums rounded once to bf16, so they may
    differ from the oracle rounded to bf16 by one bf16 unit where the fp32
    accumulation order lands on the other side of a rounding boundary: bound
    2^-8 relative per element (+1e-6 of the scale); gw (fp32, sums over
    n*h*w pixels) 2e-5 of its scale."""
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import _Conv3x3Bf16
    x, wt, gy = _case(cin, cout, n, h, w, 7 * cin + h + w)
    passes = tuple(bool(_abi.query("mde_conv3x3_supported", cin, cout, i, _abi.MDE_BF16))
                   for i in range(3))
    assert passes == (True, True, True)
    xr = _bf(x).requires_grad_(True)
    wr = _bf(wt).requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, 1)
    yr.backward(_bf(gy))
    xg = x.to(DEV, torch.bfloat16).requires_grad_(True)
    wg = wt.to(DEV).requires_grad_(True)
    y, _ = _Conv3x3Bf16.apply(xg, wg, passes, False)
    assert y.dtype == torch.bfloat16
    y.backward(gy.to(DEV, torch.bfloat16))
    assert xg.grad.dtype == torch.bfloat16 and wg.grad.dtype == torch.float32
    for got, want, what in ((y, yr, "forward"), (xg.grad, xr.grad, "data gradient")):
        g = got.detach().double().cpu()
        scale = float(want.abs().max())
        bad = (g - want).abs() > (2.0 ** -8) * want.abs() + 1e-6 * scale
        assert not bool(bad.any()), (what, float((g - want).abs().max()), scale)
    assert rel_err(wg.grad, wr.grad) <= 2e-5, "weight gradient"


@pytest.mark.parametrize("cin,cout", BF_PAIRS)
def test_conv3x3_bf16_stats_epilogue(cin, cout):
    """The bf16 forward's BatchNorm-statistics epilogue describes the bf16 y
    it wrote: merged (count, mean, M2) equal float64 statistics of y."""
    from monocular_depth_estimation_amd.nn import _Conv3x3Bf16
    x, wt, _ = _case(cin, cout, 3, 29, 100, 11 + cin)
    xg = x.to(DEV, torch.bfloat16)
    y, st = _Conv3x3Bf16.apply(xg, wt.to(DEV), (True, True, True), True)
    st = st.double().cpu()
    yd = y.double().cpu()
    for c in range(cout):
        ref, cnt, s1, s2 = st[c, :, 0], st[c, :, 1], st[c, :, 2], st[c, :, 3]
        n = float(cnt.sum())
        mean = float((s1 + cnt * ref).sum()) / n
        ex2 = float((s2 + 2 * ref * s1 + cnt * ref * ref).sum()) / n
        v = yd[:, c]
        assert n == v.numel()
        assert abs(mean - float(v.mean())) <= 1e-5 * (1 + abs(float(v.mean())))
        assert abs((ex2 - mean * mean) - float(v.var(unbiased=False))) <= 1e-4 * float(v.var())


# Stride-2 stem convolutions (DDRNet_23_slim.py:229-236): weight gradient on
# the HIP kernel vs float64; (h, w) cover full 64-column tiles (wo = 320 at
# 480x640), a ragged last tile (wo = 160 / 90), odd heights (a half-filled
# last input row) and a single output row.
S2 = [(3, 32, 2, 480, 640), (32, 32, 2, 240, 320), (32, 32, 1, 37, 180), (3, 32, 1, 9, 130),
      (32, 32, 2, 2, 64)]


@pytest.mark.parametrize("cin,cout,n,h,w", S2)
def test_conv3x3s2_wgrad_vs_float64(cin, cout, n, h, w):
    from monocular_depth_estimation_amd.nn import _Conv3x3S2
    x, wt, _ = _case(cin, cout, n, h, w, 5 * cin + h)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    gy = torch.rand((n, cout, ho, wo)) - 0.5
    xr = x.double().requires_grad_(cin != 3)
    wr = wt.double().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, None, 2, 1).backward(gy.double())
    xd = x.to(DEV).requires_grad_(cin != 3)
    wd = wt.to(DEV).requires_grad_(True)
    y = _Conv3x3S2.apply(xd, wd)
    y.backward(gy.to(DEV))
    assert rel_err(wd.grad, wr.grad) <= 2e-5
    if cin != 3:
        assert rel_err(xd.grad, xr.grad) <= 1e-5


def test_conv3x3s2_wgrad_deterministic():
    from monocular_depth_estimation_amd.nn import _Conv3x3S2
    x, wt, _ = _case(32, 32, 2, 64, 96, 4)
    gy = (torch.rand((2, 32, 32, 48)) - 0.5).to(DEV)
    outs = []
    for _ in range(2):
        wd = wt.to(DEV).requires_grad_(True)
        _Conv3x3S2.apply(x.to(DEV), wd).backward(gy)
        outs.append(wd.grad.cpu())
    assert torch.equal(outs[0], outs[1])



# Stride-2 wide weight gradients (DDRNet's stride-2 BasicBlock convs and
# down3 / down4): output widths 80 (two 40-column strips), 40, 20, a ragged
# last row tile (odd input height), and an unsupported width (MIOpen path).
S2W = [(32, 64, 2, 120, 160), (64, 128, 2, 60, 80), (128, 256, 2, 30, 40), (64, 128, 1, 37, 80)]


@pytest.mark.parametrize("cin,cout,n,h,w", S2W)
def test_conv3x3s2_wide_wgrad_vs_float64(cin, cout, n, h, w):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import _Conv3x3S2
    assert _abi.query("mde_conv3x3s2_wgrad_workspace", n, cin, cout, h, w, 0) > 0
    x, wt, _ = _case(cin, cout, n, h, w, 3 * cin + h)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    gy = torch.rand((n, cout, ho, wo)) - 0.5
    xr = x.double().requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, None, 2, 1).backward(gy.double())
    xd = x.to(DEV).requires_grad_(True)
    wd = wt.to(DEV).requires_grad_(True)
    _Conv3x3S2.apply(xd, wd).backward(gy.to(DEV))
    assert rel_err(wd.grad, wr.grad) <= 2e-5
    assert rel_err(xd.grad, xr.grad) <= 1e-5


def test_conv3x3s2_wide_unsupported_width_falls_back():
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import conv3x3s2_ok
    assert _abi.query("mde_conv3x3s2_wgrad_workspace", 2, 256, 256, 15, 20, 0) == 0  # wo = 10
    conv = torch.nn.Conv2d(256, 256, 3, 2, 1, bias=False)
    assert not conv3x3s2_ok(conv, torch.empty((2, 256, 15, 20), device=DEV))
