"""GPU parity of the wide 1x1 convolutions (mde_conv1x1_*, csrc/conv1x1.hip).

The reference layers are DDRNet-23-slim's bias-free 1x1 convs
(src/GuideDepth/model/DDRNet_23_slim.py:79,84 Bottleneck, :294-296 the
stride-2 downsample, :245,250 compression, :121-171 DAPPM); their ATen conv2d
(the reference's own dependency) evaluated in float64 on the CPU is the
oracle.  Tolerances (written per assertion): forward / data gradient 1e-5 of
the output's max magnitude (fp32 MFMA sums of <= 640 products), weight
gradient 2e-5 (fp32 sums over up to 10^6 pixels, split over blocks and
reduced in a fixed order).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
# (cin, cout, stride, h, w): every DDRNet 1x1 at its cfg2 plane size, and
# odd / ragged planes (h = 15 -> 8 rows at stride 2, pixel tiles past the plane)
SHAPES = [(32, 64, 2, 120, 160), (64, 128, 2, 60, 80), (128, 256, 2, 30, 40),
          (256, 512, 2, 15, 20), (64, 128, 1, 60, 80), (128, 64, 1, 30, 40),
          (256, 64, 1, 15, 20), (256, 256, 1, 15, 20), (256, 512, 1, 8, 10),
          (512, 128, 1, 8, 10), (640, 128, 1, 8, 10), (96, 160, 1, 6, 6),
          (64, 96, 2, 15, 20), (96, 64, 2, 13, 24),
          # MobileNetV3-Large's expand / project 1x1s (mobilenetv3.py LARGE):
          # channel counts that are multiples of 8, not 32 (padded in-kernel)
          (16, 64, 1, 24, 32), (64, 24, 1, 12, 16), (24, 72, 1, 12, 16), (72, 40, 1, 10, 12),
          (40, 120, 1, 6, 8), (240, 80, 1, 6, 8), (80, 200, 1, 6, 8), (184, 80, 1, 6, 8),
          (480, 112, 1, 5, 8), (112, 672, 1, 4, 8), (24, 40, 2, 16, 20), (40, 24, 2, 13, 24)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    import monocular_depth_estimation_amd  # noqa: F401


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("cin,cout,stride,h,w", SHAPES)
def test_conv1x1_vs_float64_oracle(cin, cout, stride, h, w):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.nn import Conv2d, conv1x1_ok
    n = 3
    g = torch.Generator().manual_seed(cin * 7 + cout + h)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin, 1, 1), generator=g) - 0.5) * 0.2
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    gy = torch.rand((n, cout, ho, wo), generator=g) - 0.5
    xr = x.double().requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, stride)
    yr.backward(gy.double())

    conv = Conv2d(cin, cout, 1, stride=stride, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
    xg = x.to(DEV).requires_grad_(True)
    assert conv1x1_ok(conv, xg)
    assert _abi.query("mde_conv1x1_supported", cin, cout, h, w, stride, 0) == 1
    y = conv(xg)  # stride 1: the MIOpen forward; HIP data / weight gradients
    yh = torch.empty_like(y)
    w2 = conv.weight.detach().reshape(cout, cin).contiguous()
    _abi.call("mde_conv1x1_fwd", _abi.ptr(xg.detach()), _abi.ptr(w2), _abi.ptr(yh), n, cin, cout,
              h, w, stride, 0, _abi.stream_of(xg))
    assert rel_err(yh, yr) <= 1e-5, "HIP forward"
    y.backward(gy.to(DEV))
    assert y.shape == yr.shape
    assert rel_err(y, yr) <= 1e-5, "forward"
    assert rel_err(xg.grad, xr.grad) <= 1e-5, "data gradient"
    assert rel_err(conv.weight.grad, wr.grad) <= 2e-5, "weight gradient"


@pytest.mark.parametrize("cin,cout,stride,h,w", [(32, 64, 2, 120, 160), (64, 128, 1, 60, 80),
                                                 (640, 128, 1, 8, 10),
                                                 # the small-channel weight-gradient path
                                                 (16, 64, 1, 240, 320), (72, 24, 1, 120, 160),
                                                 (120, 40, 1, 60, 80), (64, 64, 1, 60, 80),
                                                 # wide padded M (64-row tiles under MDE_C1_BM_AUTO=1)
                                                 (112, 672, 1, 30, 40), (480, 112, 1, 30, 40)])
def test_conv1x1_full_batch_vs_miopen_and_deterministic(cin, cout, stride, h, w):
    """cfg2 batch (32): HIP vs MIOpen fp32 on the GPU for all three passes, and
    two runs bitwise equal (the weight gradient's fixed-order reduction)."""
    from monocular_depth_estimation_amd.nn import _Conv1x1
    gen = torch.Generator(device=DEV).manual_seed(cin + cout)
    x = torch.rand((32, cin, h, w), device=DEV, generator=gen) - 0.5
    wt = (torch.rand((cout, cin, 1, 1), device=DEV, generator=gen) - 0.5) * 0.2
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    gy = torch.rand((32, cout, ho, wo), device=DEV, generator=gen) - 0.5
    outs = []
    for _ in range(2):
        xh = x.clone().requires_grad_(True)
        wh = wt.clone().requires_grad_(True)
        y = _Conv1x1.apply(xh, wh, stride)
        y.backward(gy)
        outs.append((y.detach(), xh.grad, wh.grad))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    xm = x.clone().requires_grad_(True)
    wm = wt.clone().requires_grad_(True)
    ym = torch.nn.functional.conv2d(xm, wm, None, stride)
    ym.backward(gy)
    y, gx, gw = outs[0]
    assert rel_err(y, ym) <= 2e-5
    assert rel_err(gx, xm.grad) <= 2e-5
    assert rel_err(gw, wm.grad) <= 5e-5


def test_conv1x1_small_planes_are_not_taken():
    """Planes of fewer than 32 output pixels (DAPPM's pooled 4x5 / 2x3 maps)
    stay on MIOpen: the weight gradient's pixel chunks assume a chunk touches
    at most two images."""
    from monocular_depth_estimation_amd import _abi
    assert _abi.query("mde_conv1x1_supported", 512, 128, 4, 5, 1, 0) == 0
    assert _abi.query("mde_conv1x1_supported", 512, 128, 8, 10, 1, 0) == 1
    # channel counts: multiples of 8, >= 16
    assert _abi.query("mde_conv1x1_supported", 12, 128, 8, 10, 1, 0) == 0
    assert _abi.query("mde_conv1x1_supported", 8, 128, 8, 10, 1, 0) == 0
    assert _abi.query("mde_conv1x1_supported", 16, 24, 8, 10, 1, 0) == 1


def test_conv1x1_stride2_zero_fills_odd_positions():
    """The stride-2 data gradient overwrites gx completely: zeros at every odd
    row / column (the 1x1 / s2 conv never reads them), also with a dirty buffer."""
    from monocular_depth_estimation_amd import _abi
    n, cin, cout, h, w = 2, 64, 128, 15, 20
    gy = torch.rand((n, cout, 8, 10), device=DEV) + 0.5
    wt = torch.rand((cout, cin), device=DEV) + 0.5
    gx = torch.full((n, cin, h, w), float("nan"), device=DEV)
    _abi.call("mde_conv1x1_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, cin, cout, h, w,
              2, 0, _abi.stream_of(gy))
    torch.cuda.synchronize()
    assert bool(torch.isfinite(gx).all())
    assert float(gx[:, :, 1::2, :].abs().max()) == 0.0
    assert float(gx[:, :, :, 1::2].abs().max()) == 0.0
    assert float(gx[:, :, 0::2, 0::2].min()) > 0.0


@pytest.mark.parametrize("cin,cout,h,w", [(16, 16, 10, 14), (24, 72, 7, 12), (40, 120, 9, 20),
                                          (64, 24, 4, 9), (120, 40, 5, 16)])
def test_conv1x1_mix_small_writes_every_output(cin, cout, h, w):
    """The small-channel channel mix (c1_mix_small_kernel: stride 1, K and M <=
    128 off the 32 grid; 64-pixel wave chunks, ragged at the plane's end,
    channels padded to 16-row tiles) overwrites NaN-filled outputs completely
    and matches float64 for both the forward and the data gradient."""
    from monocular_depth_estimation_amd import _abi
    n = 3
    g = torch.Generator().manual_seed(cin * cout + h)
    x = torch.rand((n, cin, h, w), generator=g) - 0.5
    wt = (torch.rand((cout, cin), generator=g) - 0.5) * 0.2
    gy = torch.rand((n, cout, h, w), generator=g) - 0.5
    yr = torch.einsum("oc,nchw->nohw", wt.double(), x.double())
    gxr = torch.einsum("oc,nohw->nchw", wt.double(), gy.double())
    xd, wd, gyd = x.to(DEV), wt.to(DEV), gy.to(DEV)
    y = torch.full((n, cout, h, w), float("nan"), device=DEV)
    gx = torch.full((n, cin, h, w), float("nan"), device=DEV)
    st = _abi.stream_of(xd)
    _abi.call("mde_conv1x1_fwd", _abi.ptr(xd), _abi.ptr(wd), _abi.ptr(y), n, cin, cout, h, w, 1, 0,
              st)
    _abi.call("mde_conv1x1_bwd_data", _abi.ptr(gyd), _abi.ptr(wd), _abi.ptr(gx), n, cin, cout, h, w,
              1, 0, st)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(y).all()) and bool(torch.isfinite(gx).all())
    assert rel_err(y, yr) <= 1e-5, "forward"
    assert rel_err(gx, gxr) <= 1e-5, "data gradient"
