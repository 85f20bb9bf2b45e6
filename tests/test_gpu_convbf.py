"""GPU parity of the bf16 implicit-GEMM convolutions (convbf.hip) through
nn.Conv2d's bf16-autocast route (_ConvBf16): forward, data gradient, weight
gradient.

Reference layers: every convolution of DDRNet-23-slim's encoder under bf16
autocast (src/GuideDepth/model/DDRNet_23_slim.py:35-38 conv3x3, :41-113
BasicBlock / Bottleneck, :121-171 DAPPM, :230-263 stem / down / compression,
the 1x1 downsamples of _make_layer :291-309).  Oracle = ATen conv2d (the
reference's own dependency) in float64 on the CPU, on the bf16-ROUNDED
operands autocast hands a conv (x, gy and the weight rounded to bf16, RNE):
what is left is the kernels' fp32 accumulation and the bf16 rounding of y /
gx.  Tolerances: y and gx within 2^-8 of each element's magnitude plus 1e-3
of the tensor's max (one bf16 rounding + fp32 sums of <= 5760 products);
the fp32 weight gradient within 1e-4 of its max magnitude.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
# (cin, cout, h, w, k, stride) input sizes: DDRNet's convs at cfg3 sizes
# (bs 2 here), plus odd heights, 2D-tile planes and the decoder-width case
SHAPES = [
    (64, 64, 60, 80, 3, 1),     # layer2 / layer3_ / layer4_ BasicBlocks
    (128, 128, 30, 40, 3, 1),   # layer3
    (256, 256, 15, 20, 3, 1),   # layer4 (odd height)
    (128, 128, 8, 10, 3, 1),    # DAPPM process (80-pixel planes)
    (128, 64, 60, 80, 3, 1),    # segmenthead conv1
    (32, 64, 120, 160, 3, 2),   # layer2 stride-2
    (64, 128, 60, 80, 3, 2),    # layer3 / down3 / down4
    (128, 256, 30, 40, 3, 2),   # layer4 / down4
    (256, 256, 15, 20, 3, 2),   # layer5 Bottleneck conv2 (odd input height)
    (32, 32, 240, 320, 3, 2),   # stem conv1[3] (32 output channels)
    (64, 64, 60, 80, 1, 1),     # Bottleneck conv1 / compression
    (64, 128, 60, 80, 1, 1),    # Bottleneck conv3 / downsample
    (512, 128, 8, 10, 1, 1),    # DAPPM scale0 / shortcut
    (640, 256, 8, 10, 1, 1),    # DAPPM compression
    (32, 64, 120, 160, 1, 2),   # layer2 downsample
    (256, 512, 15, 20, 1, 2),   # layer5 downsample (odd input height)
    (64, 32, 18, 24, 3, 1),     # 32 output channels, small plane
    (96, 64, 26, 160, 3, 2),    # 3 input-channel chunks, 2D tiles with a ragged last band
    (96, 64, 22, 40, 3, 2),     # 3 input-channel chunks, 11 x 20 output plane
]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    import monocular_depth_estimation_amd  # noqa: F401


def _bf(t):
    return t.to(torch.bfloat16).double()


def _close(got, ref, rel=2.0 ** -8, frac=1e-3):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    bound = rel * ref.abs() + frac * ref.abs().max()
    bad = (got - ref).abs() > bound
    return int(bad.sum()), float(((got - ref).abs() / ref.abs().max()).max())


@pytest.mark.parametrize("cin,cout,h,w,k,s", SHAPES)
def test_convbf_vs_float64_oracle(cin, cout, h, w, k, s):
    from monocular_depth_estimation_amd.nn import Conv2d, convbf_ok
    n = 2
    g = torch.Generator().manual_seed(cin + 7 * cout + h + 13 * k + s)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = torch.randn((cout, cin, k, k), generator=g) * (2.0 / (cin * k * k)) ** 0.5
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
    gy = torch.rand((n, cout, ho, wo), generator=g) - 0.5
    xr = _bf(x).requires_grad_(True)
    wr = _bf(wt).requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, s, pad)
    yr.backward(_bf(gy))
    conv = Conv2d(cin, cout, k, stride=s, padding=pad, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
    xg = x.to(DEV).to(torch.bfloat16).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        assert convbf_ok(conv, xg)
        y = conv(xg)
    assert y.dtype == torch.bfloat16 and y.shape == yr.shape
    y.backward(gy.to(DEV).to(torch.bfloat16))
    torch.cuda.synchronize()
    nbad, worst = _close(y, yr)
    assert nbad == 0, f"forward: {nbad} elements out of tolerance (worst {worst:.2e})"
    assert xg.grad.dtype == torch.bfloat16
    nbad, worst = _close(xg.grad, xr.grad)
    assert nbad == 0, f"data gradient: {nbad} elements out of tolerance (worst {worst:.2e})"
    assert conv.weight.grad.dtype == torch.float32
    gw, gwr = conv.weight.grad.double().cpu(), wr.grad
    err = float((gw - gwr).abs().max() / gwr.abs().max())
    assert err <= 1e-4, f"weight gradient rel err {err:.2e}"


def test_convbf_weight_gradient_is_deterministic():
    """Fixed-order split-K reduction: two runs are bitwise equal."""
    from monocular_depth_estimation_amd.nn import Conv2d
    conv = Conv2d(64, 64, 3, padding=1, bias=False).to(DEV)
    x = torch.randn((4, 64, 60, 80), device=DEV).to(torch.bfloat16)
    gy = torch.randn((4, 64, 60, 80), device=DEV).to(torch.bfloat16)
    grads = []
    for _ in range(2):
        conv.weight.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            y = conv(x)
        y.backward(gy)
        grads.append(conv.weight.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_convbf_pack_scope_matches_per_conv_pack():
    """convbf_pack_scope (every filter packed by one table launch) gives
    bitwise the outputs and gradients of the per-conv pack, across weight
    updates and a conv registered late."""
    from monocular_depth_estimation_amd import nn as mnn
    from monocular_depth_estimation_amd.nn import Conv2d

    class Two(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Conv2d(64, 128, 3, stride=2, padding=1, bias=False)
            self.b = Conv2d(128, 64, 1, bias=False)
            self.c = Conv2d(64, 64, 3, padding=1, bias=False)

        def forward(self, x, late):
            y = self.b(self.a(x))
            return self.c(y) if late else y

    m = Two().to(DEV)
    x = torch.randn((2, 64, 60, 80), device=DEV).to(torch.bfloat16)

    def run(scoped, late):
        xg = x.clone().requires_grad_(True)
        for p in m.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            if scoped:
                with mnn.convbf_pack_scope(m, x.device):
                    y = m(xg, late)
            else:
                y = m(xg, late)
        y.float().square().sum().backward()
        return [y.detach().clone(), xg.grad.clone()] + [p.grad.clone() for p in m.parameters()
                                                        if p.grad is not None]

    for step in range(4):
        late = step >= 2
        got, ref = run(True, late), run(False, late)
        assert len(got) == len(ref)
        for g_, r_ in zip(got, ref):
            assert torch.equal(g_, r_), f"step {step}"
        sc = m.__dict__["_convbf_pack"]
        assert len(sc.entries) == (3 if late else 2)
        if step >= 1:
            assert len(sc.packed) == (2 if step == 2 else len(sc.entries))
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(0.9).add_(0.01)


def test_convbf_pack_scope_survives_rebuild_after_capture():
    """a captured forward records the pack table's device pointer.
    An eager forward after the capture that registers a new conv rebuilds the
    table; the old one must stay alive (the scope keeps retired tables), so
    the graph's replays still pack every filter it uses: replayed outputs ==
    eager outputs at the same weights, before and after the rebuild."""
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd import nn as mnn
    from monocular_depth_estimation_amd.nn import Conv2d

    class Two(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Conv2d(64, 128, 3, stride=2, padding=1, bias=False)
            self.b = Conv2d(128, 64, 1, bias=False)
            self.c = Conv2d(64, 64, 3, padding=1, bias=False)

        def forward(self, x, late):
            y = self.b(self.a(x))
            return self.c(y) if late else y

    m = Two().to(DEV)
    x = torch.randn((2, 64, 60, 80), device=DEV).to(torch.bfloat16)
    out = torch.empty((2, 64, 30, 40), device=DEV, dtype=torch.bfloat16)

    def fwd(late):
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            with mnn.convbf_pack_scope(m, x.device):
                return m(x, late)

    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fwd(False)  # registers a, b
            fwd(False)  # they are in the table from here
        torch.cuda.current_stream().wait_stream(s)
        g, _, _ = _abi.capture_graph(lambda: out.copy_(fwd(False)), s)
        sc = m.__dict__["_convbf_pack"]
        table0 = sc.table
        for p in m.parameters():
            p.mul_(0.9).add_(0.01)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, fwd(False))
        fwd(True)  # registers c: the next forward rebuilds the table
        fwd(True)
        assert sc.table is not table0 and any(t is table0 for t in sc.retired)
        torch.cuda.empty_cache()
        for p in m.parameters():
            p.mul_(0.9).add_(0.01)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, fwd(False))
    g.reset()


def test_convbf_biased_conv_adds_bias_in_bf16():
    """Conv2d(bias=True) on the bf16 route (DDRNet's segmenthead 1x1): output in
    autocast's dtype, bias gradient = the sum of gy."""
    from monocular_depth_estimation_amd.nn import Conv2d
    conv = Conv2d(64, 64, 1, bias=True).to(DEV)
    x = torch.randn((2, 64, 60, 80), device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y = conv(x)
    assert y.dtype == torch.bfloat16
    gy = torch.randn_like(y)
    y.backward(gy)
    ref = gy.double().sum((0, 2, 3))
    err = float((conv.bias.grad.double() - ref).abs().max() / ref.abs().max())
    assert err <= 1e-2, err


def test_convbf_refuses_unaligned_planes():
    """Output planes whose pixel count breaks the 4-pixel store groups (and
    whose width is not a multiple of 4) are not taken: MIOpen runs them."""
    from monocular_depth_estimation_amd import _abi
    assert _abi.query("mde_convbf_supported", 96, 64, 22, 36, 3, 2, 0) == 0  # 11 x 18 output
    assert _abi.query("mde_convbf_supported", 96, 64, 22, 40, 3, 2, 0) == 1


@pytest.mark.parametrize("cin,cout,h,w,k,s", [
    (64, 64, 60, 80, 3, 1), (128, 64, 60, 80, 3, 1), (32, 64, 120, 160, 3, 2),
    (256, 256, 15, 20, 3, 2), (32, 64, 120, 160, 1, 2), (640, 256, 8, 10, 1, 1),
    (64, 32, 18, 24, 3, 1),
])
def test_convbf_epilogue_statistics(cin, cout, h, w, k, s):
    """The forward's per-block BN sums [cout][blocks][4] (shift, count, s1, s2)
    merge to the mean / variance of the bf16 y it wrote (float64 reference)."""
    from monocular_depth_estimation_amd.nn import Conv2d, conv_bf16_stats
    n = 4
    torch.manual_seed(cin + cout + k)
    conv = Conv2d(cin, cout, k, stride=s, padding=k // 2, bias=False).to(DEV)
    x = (torch.rand((n, cin, h, w), device=DEV) - 0.3).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y, st = conv_bf16_stats(conv, x)
    torch.cuda.synchronize()
    assert st is not None and st.shape[0] == cout
    st = st.double().cpu()
    ref, cnt, s1, s2 = st[..., 0], st[..., 1], st[..., 2], st[..., 3]
    tot = cnt.sum(1)
    assert torch.all(tot == n * y.shape[2] * y.shape[3])
    mean = (ref * cnt + s1).sum(1) / tot
    ex2 = (s2 + 2 * ref * s1 + cnt * ref * ref).sum(1) / tot
    var = ex2 - mean * mean
    yd = y.double().cpu()
    mref = yd.mean((0, 2, 3))
    vref = yd.var((0, 2, 3), unbiased=False)
    scale = yd.abs().max()
    assert float((mean - mref).abs().max() / scale) < 1e-5
    assert float(((var - vref).abs() / vref).max()) < 1e-3


@pytest.mark.parametrize("cin,cout,h,w,k,s", [(64, 64, 60, 80, 3, 1), (32, 64, 120, 160, 1, 2)])
def test_batchnorm_from_convbf_records_matches_statistics_pass(cin, cout, h, w, k, s):
    """BatchNorm (train) fed the conv epilogue's records -- merged by the
    plane-mode apply itself (mde_batchnorm_stats_route 1) -- against the same
    BatchNorm taking its own statistics pass: outputs within one bf16 ulp,
    running statistics and saved moments within 1e-5."""
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import BatchNorm2d, Conv2d, batch_norm_act, conv_bf16_stats
    n = 8
    torch.manual_seed(3)
    conv = Conv2d(cin, cout, k, stride=s, padding=k // 2, bias=False).to(DEV)
    x = torch.randn((n, cin, h, w), device=DEV).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y, st = conv_bf16_stats(conv, x)
    assert st is not None
    ho, wo = y.shape[2], y.shape[3]
    assert _abi.query("mde_batchnorm_stats_route", n, cout, ho, wo, st.shape[1], _abi.MDE_BF16) == 1
    gamma = torch.rand(cout, device=DEV) + 0.5
    beta = torch.rand(cout, device=DEV) * 0.4 - 0.2
    outs = []
    for stats in (st, None):
        bn = BatchNorm2d(cout, act="relu").to(DEV)
        with torch.no_grad():
            bn.weight.copy_(gamma)
            bn.bias.copy_(beta)
            out = batch_norm_act(y.detach(), bn, "relu", None, None, stats)
        outs.append((out.float(), bn.running_mean.clone(), bn.running_var.clone()))
    torch.cuda.synchronize()
    (a, ma, va), (b, mb, vb) = outs
    ulp = 2.0 ** -7 * b.abs().clamp_min(2.0 ** -14)
    assert bool(((a - b).abs() <= ulp).all())
    assert float((ma - mb).abs().max()) < 1e-5 and float(((va - vb).abs() / vb).max()) < 1e-5
