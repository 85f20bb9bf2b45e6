"""GPU parity of the Winograd F(2x2, 3x3) stride-1 convolutions (wino.hip):
forward and data gradient of DDRNet's wide 3x3 convs (src/GuideDepth/model/
DDRNet_23_slim.py:41-72 BasicBlocks, :121-171 DAPPM, :201-210 seg head).

Oracle: ATen conv2d (the reference's own dependency) in float64 on the CPU.
Tolerance (per assertion): 1e-5 of the output's max magnitude -- the
transforms are exact up to fp32 rounding (B^T / A^T entries 0, +-1; G's
0, +-1/2) and the GEMMs sum <= 16 * 256 fp32 products.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
# (cin, cout, h, w): the cfg2 shapes (bs 2), ragged planes (partial 8 x 16
# blocks: 15 / 9 / 11 rows, 20 / 40 / 30 / 18 columns), 32- and 64-channel
# output groups, 16 -> 16 (16-channel groups, 8 x 32-pixel blocks), cin = 16
# (one channel chunk)
SHAPES = [(32, 32, 120, 160), (64, 64, 60, 80), (128, 128, 30, 40), (256, 256, 15, 20),
          (128, 64, 60, 80), (64, 128, 60, 80), (64, 64, 9, 40), (128, 64, 11, 30),
          (16, 32, 10, 18), (32, 96, 7, 34), (16, 16, 40, 70)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    import monocular_depth_estimation_amd  # noqa: F401


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("cin,cout,h,w", SHAPES)
def test_wino_abi_vs_float64_oracle(cin, cout, h, w):
    """Both passes through the C ABI: the forward transform + conv, and the
    flipped transform + conv of gy (the data gradient)."""
    from monocular_depth_estimation_amd import _abi
    n = 2
    g = torch.Generator().manual_seed(cin + 3 * cout + h + w)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), generator=g) - 0.5) * 0.1
    gy = torch.rand((n, cout, h, w), generator=g) - 0.5
    xr = x.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wt.double(), None, 1, 1)
    yr.backward(gy.double())
    assert _abi.query("mde_wino_supported", cin, cout, h, w, 0) == 1
    assert _abi.query("mde_wino_supported", cout, cin, h, w, 0) == 1
    xd, wd, gyd = x.to(DEV), wt.to(DEV), gy.to(DEV)
    st = _abi.stream_of(xd)
    u = torch.empty(_abi.query("mde_wino_weight_bytes", cin, cout) // 4, device=DEV)
    y = torch.full((n, cout, h, w), float("nan"), device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wd), _abi.ptr(u), cin, cout, 0, st)
    _abi.call("mde_wino_conv", _abi.ptr(xd), _abi.ptr(u), _abi.ptr(y), n, cin, cout, h, w, 0, 0, st)
    assert rel_err(y, yr) <= 1e-5, "forward"
    gx = torch.full_like(xd, float("nan"))
    _abi.call("mde_wino_weight", _abi.ptr(wd), _abi.ptr(u), cin, cout, 1, st)
    _abi.call("mde_wino_conv", _abi.ptr(gyd), _abi.ptr(u), _abi.ptr(gx), n, cout, cin, h, w, 1, 0,
              st)
    assert rel_err(gx, xr.grad) <= 1e-5, "data gradient"


@pytest.mark.parametrize("cin,cout,h,w", [(64, 64, 60, 80), (128, 64, 60, 80), (256, 256, 15, 20)])
def test_wino_module_path(cin, cout, h, w, monkeypatch):
    """Conv2d (the DDRNet modules' class) dispatches both passes to Winograd
    at cfg2 sizes (bs 16: >= 256 blocks of 8 x 16 pixels x 64 channels) with
    MDE_WINO on; all three gradients vs float64."""
    from monocular_depth_estimation_amd import nn as mnn
    from monocular_depth_estimation_amd.nn import WINO, Conv2d, conv3x3_passes
    monkeypatch.setattr(mnn, "WINO_ON", True)
    n = 16
    g = torch.Generator().manual_seed(cin * 11 + cout)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), generator=g) - 0.5) * 0.1
    gy = torch.rand((n, cout, h, w), generator=g) - 0.5
    xr = x.double().requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, 1)
    yr.backward(gy.double())
    conv = Conv2d(cin, cout, 3, padding=1, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
    xg = x.to(DEV).requires_grad_(True)
    passes = conv3x3_passes(conv, xg)
    assert passes is not None and passes[0] == WINO and passes[1] == WINO, passes
    y = conv(xg)
    y.backward(gy.to(DEV))
    assert rel_err(y, yr) <= 1e-5, "forward"
    assert rel_err(xg.grad, xr.grad) <= 1e-5, "data gradient"
    assert rel_err(conv.weight.grad, wr.grad) <= 2e-5, "weight gradient"


def test_wino_deterministic_full_batch():
    """cfg2 batch (32) of the 64 -> 64 BasicBlock conv: two runs bitwise equal
    (no atomics; fixed summation order) and within 2e-5 of MIOpen fp32."""
    from monocular_depth_estimation_amd import _abi
    gen = torch.Generator(device=DEV).manual_seed(3)
    x = torch.rand((32, 64, 60, 80), device=DEV, generator=gen) - 0.5
    wt = (torch.rand((64, 64, 3, 3), device=DEV, generator=gen) - 0.5) * 0.1
    st = _abi.stream_of(x)
    u = torch.empty(16 * 64 * 64, device=DEV)
    outs = []
    for _ in range(2):
        y = torch.empty_like(x)
        _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), 64, 64, 0, st)
        _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y), 32, 64, 64, 60, 80, 0, 0,
                  st)
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    assert rel_err(outs[0], torch.nn.functional.conv2d(x, wt, None, 1, 1)) <= 2e-5


@pytest.mark.parametrize("cin,cout,h,w", [(16, 16, 40, 64), (64, 64, 15, 20), (32, 32, 9, 36),
                                          (64, 256, 15, 20)])  # the last: XCD split 4
def test_wino_stats_epilogue(cin, cout, h, w):
    """The BN-statistics epilogue: per (channel, pixel block) (shift, count,
    s1, s2) records whose merge gives y's batch mean / variance (float64
    recomputation from y; rel 1e-5), and y identical to the plain launch."""
    from monocular_depth_estimation_amd import _abi
    n = 3
    gen = torch.Generator(device=DEV).manual_seed(cin + h)
    x = torch.rand((n, cin, h, w), device=DEV, generator=gen) + 0.5  # offset mean
    wt = (torch.rand((cout, cin, 3, 3), device=DEV, generator=gen) - 0.4) * 0.2
    st = _abi.stream_of(x)
    u = torch.empty(16 * cin * cout, device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), cin, cout, 0, st)
    nb = _abi.query("mde_wino_stats_blocks", n, cin, cout, h, w)
    assert nb == n * -(-h // 8) * -(-w // (32 if cout == 16 else 16))
    stats = torch.full((cout, nb, 4), float("nan"), device=DEV)
    y = torch.empty((n, cout, h, w), device=DEV)
    y2 = torch.empty_like(y)
    _abi.call("mde_wino_conv_stats", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y), _abi.ptr(stats), n, cin,
              cout, h, w, 0, 0, st)
    _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y2), n, cin, cout, h, w, 0, 0, st)
    assert torch.equal(y, y2)
    s = stats.double().cpu()
    ref, cnt, s1, s2 = s[..., 0], s[..., 1], s[..., 2], s[..., 3]
    assert float(cnt.sum(1).min()) == n * h * w
    mean = (s1 + cnt * ref).sum(1) / cnt.sum(1)
    ex2 = (s2 + 2 * ref * s1 + cnt * ref * ref).sum(1) / cnt.sum(1)
    var = ex2 - mean * mean
    yd = y.double().cpu()
    mr = yd.mean((0, 2, 3))
    vr = yd.var((0, 2, 3), unbiased=False)
    assert float((mean - mr).abs().max() / mr.abs().max()) <= 1e-5
    assert float((var - vr).abs().max() / vr.abs().max()) <= 1e-4


def test_wino_weight2_matches_both_transforms():
    """mde_wino_weight2 (the forward's U and the data gradient's flipped U' in
    one launch) == mde_wino_weight with flip 0 / 1, bitwise."""
    from monocular_depth_estimation_amd import _abi

    def pad_co(c):
        return 16 if c == 16 else -(-c // 32) * 32

    def pad_ci(c):
        return -(-c // 16) * 16

    for cin, cout in ((64, 128), (32, 32), (16, 48), (24, 128), (112, 40)):
        wt = torch.rand((cout, cin, 3, 3), device=DEV) - 0.5
        st = _abi.stream_of(wt)
        nb = _abi.query("mde_wino_weight_bytes", cin, cout) // 4
        ef = 16 * pad_co(cout) * pad_ci(cin)  # the forward's padded U
        eb = 16 * pad_co(cin) * pad_ci(cout)  # the data gradient's
        assert nb == max(ef, eb)
        u0, u1, v0, v1 = (torch.full((nb,), float("nan"), device=DEV) for _ in range(4))
        _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u0), cin, cout, 0, st)
        _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u1), cin, cout, 1, st)
        _abi.call("mde_wino_weight2", _abi.ptr(wt), _abi.ptr(v0), _abi.ptr(v1), cin, cout, st)
        assert torch.equal(u0[:ef], v0[:ef]) and torch.equal(u1[:eb], v1[:eb])
        assert torch.isfinite(v0[:ef]).all() and torch.isfinite(v1[:eb]).all()
        if ef < nb:  # nothing written past the extent
            assert torch.isnan(v0[ef:]).all()
        if eb < nb:
            assert torch.isnan(v1[eb:]).all()


def test_wino_weight_table_matches_weight2():
    """mde_wino_weight_table (every conv's transforms in ONE launch, rows of
    mixed shapes, some forward-only) == mde_wino_weight2 / mde_wino_weight per
    conv, bitwise, nothing written past each extent."""
    from monocular_depth_estimation_amd import _abi
    shapes = ((64, 128, 1), (32, 32, 1), (16, 48, 0), (24, 128, 1), (112, 40, 1), (16, 16, 0),
              (128, 64, 1))
    rows, blk, pairs, bufs = [], 0, 0, []
    for cin, cout, both in shapes:
        wt = torch.rand((cout, cin, 3, 3), device=DEV) - 0.5
        nb = _abi.query("mde_wino_weight_bytes", cin, cout) // 4
        u, u2 = (torch.full((nb,), float("nan"), device=DEV) for _ in range(2))
        bufs.append((wt, u, u2, cin, cout, both, nb))
        rows.append([wt.data_ptr(), u.data_ptr(), u2.data_ptr() if both else 0, cin, cout, blk, 0, 0])
        blk += _abi.query("mde_wino_weight_blocks", cin, cout, both)
        pairs += cin * cout
    tab = torch.tensor(rows, dtype=torch.int64, device=DEV)
    _abi.call("mde_wino_weight_table", _abi.ptr(tab), len(rows), blk, pairs, _abi.stream_of(tab))
    for wt, u, u2, cin, cout, both, nb in bufs:
        st = _abi.stream_of(wt)
        v0, v1 = (torch.full((nb,), float("nan"), device=DEV) for _ in range(2))
        _abi.call("mde_wino_weight2", _abi.ptr(wt), _abi.ptr(v0), _abi.ptr(v1), cin, cout, st)
        assert torch.equal(torch.nan_to_num(u, 7.0), torch.nan_to_num(v0, 7.0)), (cin, cout)
        if both:
            assert torch.equal(torch.nan_to_num(u2, 7.0), torch.nan_to_num(v1, 7.0)), (cin, cout)
        else:
            assert torch.isnan(u2).all()


def test_wino_pack_scope_reuses_table_transforms():
    """GuideDepth fp32 under convbf_pack_scope: after the first (registering)
    forward, every Winograd conv's U / U' come from the scope's one table
    launch; they equal the per-conv transforms of the current weights after
    an optimizer update (bitwise), and the forward matches MDE_WINO_TABLE=0's."""
    from monocular_depth_estimation_amd import GuideDepth, _abi
    from monocular_depth_estimation_amd import nn as mnn
    torch.manual_seed(0)
    model = GuideDepth(pretrained=False).to(DEV)
    x = torch.rand((4, 3, 480, 640), device=DEV)  # planes large enough for Winograd
    model(x).sum().backward()  # registers
    sc = model.__dict__["_convbf_pack"]
    assert len(sc.wino) >= 6, len(sc.wino)  # 8 at bs 4 (27 at cfg2 bs 32)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(0.01 * torch.randn_like(p))
    y1 = model(x)
    assert sc.wino_packed == frozenset(sc.wino)
    torch.cuda.synchronize()
    def pad_co(c):
        return 16 if c == 16 else -(-c // 32) * 32

    def pad_ci(c):
        return -(-c // 16) * 16

    for wgt, (u, uf, cin, cout) in sc.wino.items():
        nb = u.numel()
        v0, v1 = (torch.zeros((nb,), device=DEV) for _ in range(2))
        _abi.call("mde_wino_weight2", _abi.ptr(wgt.detach()), _abi.ptr(v0), _abi.ptr(v1), cin, cout,
                  _abi.stream_of(v0))
        ef = 16 * pad_co(cout) * pad_ci(cin)  # the extents the transforms write
        eb = 16 * pad_co(cin) * pad_ci(cout)
        assert torch.equal(u[:ef], v0[:ef]), (cin, cout)
        if uf is not None:
            assert torch.equal(uf[:eb], v1[:eb]), (cin, cout)
    old = mnn.WINO_TABLE
    try:
        mnn.WINO_TABLE = False
        y0 = model(x)
    finally:
        mnn.WINO_TABLE = old
    # (the transforms are bitwise equal above; the rest of the step is not
    # bitwise run-to-run everywhere -- MIOpen's stem conv, BN statistics)
    # (measured: 8e-6 abs, the step's run-to-run noise level)
    torch.testing.assert_close(y0, y1, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cin,cout,h,w,n", [(160, 1024, 15, 20, 16), (112, 512, 30, 40, 16),
                                            (64, 128, 120, 160, 16), (24, 128, 120, 160, 2),
                                            (40, 256, 60, 80, 8)])
def test_wino_biased_conv_newcrf_projections(cin, cout, h, w, n):
    """The NewCRF projections (newcrf_layers.py NewCRF.proj_x / proj_v: 3x3
    convs WITH a bias, cfg4 bs 16) through nn.Conv2d's biased HIP path: the
    Winograd forward and data gradient (24 / 40 / 112 channels padded to the
    next 16 / 32), + bias, the weight gradient on the HIP wide kernel (24 / 40
    / 112 input channels padded to the next 32 since round 6); output and all
    three gradients vs float64."""
    from monocular_depth_estimation_amd.nn import WINO, Conv2d, conv3x3_passes
    g = torch.Generator().manual_seed(cin + cout + h)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), generator=g) - 0.5) * 0.05
    b = torch.rand((cout,), generator=g) - 0.5
    gy = torch.rand((n, cout, h, w), generator=g) - 0.5
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, wt, b))
    torch.nn.functional.conv2d(xr, wr, br, 1, 1).backward(gy.double())
    conv = Conv2d(cin, cout, 3, padding=1).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
        conv.bias.copy_(b)
    xg = x.to(DEV).requires_grad_(True)
    passes = conv3x3_passes(conv, xg)
    assert passes is not None and passes[0] == WINO, passes
    assert passes[1] == WINO, passes  # 112 -> padded to 128 output channels since round 6
    # the weight gradient on the NCHW HIP wide kernel (MDE_WIDE_WGRAD; padded
    # input channels: MDE_WIDE_PAD), the mixed-pass biased conv
    assert bool(passes[2]), passes
    y = conv(xg)
    yr = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), 1, 1)
    assert rel_err(y, yr) <= 1e-5, "forward"
    y.backward(gy.to(DEV))
    assert rel_err(xg.grad, xr.grad) <= 1e-5, "data gradient"
    assert rel_err(conv.weight.grad, wr.grad) <= 2e-5, "weight gradient"
    assert rel_err(conv.bias.grad, br.grad) <= 1e-5, "bias gradient"


@pytest.mark.parametrize("cin,cout,h,w,n", [(32, 32, 120, 160, 3), (64, 64, 60, 80, 5),
                                            (128, 128, 30, 40, 4), (256, 256, 15, 20, 3),
                                            (64, 64, 9, 40, 3), (128, 64, 11, 30, 2),
                                            (16, 32, 10, 18, 3), (32, 96, 7, 34, 2),
                                            (16, 16, 40, 70, 2), (64, 256, 15, 20, 3)])
def test_wino_persistent_bitwise(cin, cout, h, w, n):
    """The persistent kernel (mde_wino_mode 1, opt-in: blocks walk runs of tile blocks
    with one chunk pipeline across them, buffer loads, interior fast stores)
    computes the same products in the same order as the one-block-per-item
    kernel (mode 0, the default): y and the BN-statistics records bitwise equal, ragged
    planes (edge blocks) and several run lengths (MDE_WINO_IPB is the
    override; here the default split at small and large item counts)."""
    from monocular_depth_estimation_amd import _abi
    gen = torch.Generator(device=DEV).manual_seed(7 * cin + cout + h)
    x = torch.rand((n, cin, h, w), device=DEV, generator=gen) - 0.3
    wt = (torch.rand((cout, cin, 3, 3), device=DEV, generator=gen) - 0.5) * 0.1
    st = _abi.stream_of(x)
    u = torch.empty(16 * cin * cout, device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), cin, cout, 0, st)
    nb = _abi.query("mde_wino_stats_blocks", n, cin, cout, h, w)
    outs = {}
    prev = _abi.query("mde_wino_mode", -1)
    try:
        for mode in (0, 1, 2):
            _abi.query("mde_wino_mode", mode)
            y = torch.full((n, cout, h, w), float("nan"), device=DEV)
            y2 = torch.full_like(y, float("nan"))
            stats = torch.full((cout, nb, 4), float("nan"), device=DEV)
            _abi.call("mde_wino_conv_stats", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y), _abi.ptr(stats),
                      n, cin, cout, h, w, 0, 0, st)
            _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y2), n, cin, cout, h, w, 1,
                      0, st)
            torch.cuda.synchronize()
            outs[mode] = (y, y2, stats)
    finally:
        _abi.query("mde_wino_mode", prev)
    assert prev & 3 == 2  # the default: one-block kernel, B prefetch on
    for m in (1, 2):  # 2: the one-block kernel with its B operands read a step ahead
        for a, b in zip(outs[0], outs[m]):
            assert torch.equal(a, b), m
    assert torch.isfinite(outs[1][0]).all() and torch.isfinite(outs[1][2]).all()


@pytest.mark.parametrize("cin,cout,h,w,n", [(32, 32, 120, 160, 2), (64, 32, 60, 80, 3),
                                            (32, 32, 9, 36, 3), (16, 32, 10, 18, 3),
                                            (32, 96, 7, 34, 2)])
def test_wino_position_split_vs_float64(cin, cout, h, w, n):
    """wino_f23x_kernel (mode bit 4: the 32-channel blocks with the transform
    positions split across waves, the two A^T M A halves summed) against the
    float64 conv (1e-5 of max) and against the one-wave transform (2e-6 of
    max: the same products, the halves added in another order); its BN
    records merge to y's statistics like the tile-split kernel's."""
    from monocular_depth_estimation_amd import _abi
    gen = torch.Generator().manual_seed(cin * 5 + cout + w)
    x = torch.rand((n, cin, h, w), generator=gen) - 0.4
    wt = (torch.rand((cout, cin, 3, 3), generator=gen) - 0.5) * 0.1
    yr = torch.nn.functional.conv2d(x.double(), wt.double(), None, 1, 1)
    xd, wd = x.to(DEV), wt.to(DEV)
    st = _abi.stream_of(xd)
    u = torch.empty(16 * cin * cout, device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wd), _abi.ptr(u), cin, cout, 0, st)
    nb = _abi.query("mde_wino_stats_blocks", n, cin, cout, h, w)
    outs = {}
    prev = _abi.query("mde_wino_mode", -1)
    try:
        for mode in (2, 6):
            _abi.query("mde_wino_mode", mode)
            y = torch.full((n, cout, h, w), float("nan"), device=DEV)
            y2 = torch.full_like(y, float("nan"))
            stats = torch.full((cout, nb, 4), float("nan"), device=DEV)
            _abi.call("mde_wino_conv_stats", _abi.ptr(xd), _abi.ptr(u), _abi.ptr(y), _abi.ptr(stats),
                      n, cin, cout, h, w, 0, 0, st)
            _abi.call("mde_wino_conv", _abi.ptr(xd), _abi.ptr(u), _abi.ptr(y2), n, cin, cout, h, w,
                      0, 0, st)
            torch.cuda.synchronize()
            outs[mode] = (y, y2, stats)
    finally:
        _abi.query("mde_wino_mode", prev)
    y, y2, stats = outs[6]
    assert torch.equal(y, y2)
    assert rel_err(y, yr) <= 1e-5
    assert rel_err(y, outs[2][0]) <= 2e-6
    s = stats.double().cpu()
    ref, cnt, s1, s2 = s[..., 0], s[..., 1], s[..., 2], s[..., 3]
    assert float(cnt.sum(1).min()) == n * h * w
    mean = (s1 + cnt * ref).sum(1) / cnt.sum(1)
    yd = y.double().cpu()
    mr = yd.mean((0, 2, 3))
    assert float((mean - mr).abs().max() / mr.abs().max()) <= 1e-5


@pytest.mark.parametrize("cin,cout,h,w", [(32, 32, 120, 160), (64, 64, 9, 40), (128, 64, 11, 30),
                                          (64, 64, 60, 80)])
def test_wino_conv_acc_is_conv_plus_add(cin, cout, h, w):
    """mde_wino_conv_acc (the data gradient with the residual path's gradient
    summed in the epilogue) == mde_wino_conv + add bitwise: one fp32 add per
    element, as autograd's accumulation; ragged planes and both kernels."""
    from monocular_depth_estimation_amd import _abi
    n = 2
    gen = torch.Generator(device=DEV).manual_seed(cin + w)
    x = torch.rand((n, cin, h, w), device=DEV, generator=gen) - 0.5
    wt = (torch.rand((cout, cin, 3, 3), device=DEV, generator=gen) - 0.5) * 0.1
    add = torch.rand((n, cout, h, w), device=DEV, generator=gen) - 0.5
    st = _abi.stream_of(x)
    u = torch.empty(16 * cin * cout, device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), cin, cout, 0, st)
    prev = _abi.query("mde_wino_mode", -1)
    try:
        for mode in (2, 0, 1, 6):
            _abi.query("mde_wino_mode", mode)
            y = torch.empty((n, cout, h, w), device=DEV)
            ya = torch.full_like(y, float("nan"))
            _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y), n, cin, cout, h, w, 1,
                      0, st)
            _abi.call("mde_wino_conv_acc", _abi.ptr(x), _abi.ptr(u), _abi.ptr(add), _abi.ptr(ya), n,
                      cin, cout, h, w, 1, 0, st)
            assert torch.equal(ya, add + y), mode
    finally:
        _abi.query("mde_wino_mode", prev)



@pytest.mark.parametrize("cin,cout,h,w", [(24, 128, 40, 48), (40, 256, 30, 40), (128, 24, 40, 48),
                                          (256, 40, 30, 40), (512, 112, 15, 20), (24, 32, 9, 18),
                                          (40, 64, 11, 30)])
def test_wino_padded_channels_vs_float64(cin, cout, h, w):
    """Channel counts off the 16 / 32 grid (the NewCRF proj_x convs 24 -> 128,
    40 -> 256 and their data gradients 128 -> 24, 256 -> 40, 512 -> 112;
    newcrf_layers.py:384-392): input channels padded to 16 (zero planes),
    output channels to 32 (zero filter rows, not stored) -- y vs float64 at
    1e-5 of max, the output tensor untouched past its real channels (the
    buffer is exactly [n, cout, h, w]: a stray padded store would land in the
    guard region after it), the statistics records merge to y's mean."""
    from monocular_depth_estimation_amd import _abi
    n = 2
    assert _abi.query("mde_wino_supported", cin, cout, h, w, 0) == 1
    gen = torch.Generator().manual_seed(cin * 3 + cout + h)
    x = torch.rand((n, cin, h, w), generator=gen) - 0.3
    wt = (torch.rand((cout, cin, 3, 3), generator=gen) - 0.5) * 0.1
    yr = torch.nn.functional.conv2d(x.double(), wt.double(), None, 1, 1)
    xd, wd = x.to(DEV), wt.to(DEV)
    st = _abi.stream_of(xd)
    u = torch.empty(_abi.query("mde_wino_weight_bytes", cin, cout) // 4, device=DEV)
    _abi.call("mde_wino_weight", _abi.ptr(wd), _abi.ptr(u), cin, cout, 0, st)
    guard = 4096
    buf = torch.full((n * cout * h * w + guard,), float("nan"), device=DEV)
    y = buf[:n * cout * h * w].view(n, cout, h, w)
    nb = _abi.query("mde_wino_stats_blocks", n, cin, cout, h, w)
    stats = torch.full((cout, nb, 4), float("nan"), device=DEV)
    _abi.call("mde_wino_conv_stats", _abi.ptr(xd), _abi.ptr(u), _abi.ptr(y), _abi.ptr(stats), n, cin,
              cout, h, w, 0, 0, st)
    torch.cuda.synchronize()
    assert rel_err(y, yr) <= 1e-5
    assert torch.isnan(buf[n * cout * h * w:]).all()
    s = stats.double().cpu()
    ref, cnt, s1 = s[..., 0], s[..., 1], s[..., 2]
    mean = (s1 + cnt * ref).sum(1) / cnt.sum(1)
    mr = y.double().cpu().mean((0, 2, 3))
    assert float((mean - mr).abs().max() / mr.abs().max()) <= 1e-5
