"""The one-output-channel 3x3 conv (csrc/head.hip): the NewCRF depth head
(src/model_mobileV3_large_newCRFs.py Decoder.conv1 = nn.Conv2d(128, 1, 3,
padding=1)) through nn.py's Conv2d -- output, data / weight / bias gradients
vs float64 ATen conv2d on the CPU (rel. 1e-5; the weight gradient 2e-5: fp32
sums over n h w pixels in row slices, reduced in a fixed order); bitwise run
to run."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _run(x, wt, b, gy):
    from monocular_depth_estimation_amd.nn import Conv2d, head_conv_ok
    conv = Conv2d(x.shape[1], 1, 3, padding=1).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
        conv.bias.copy_(b)
    xg = x.to(DEV).requires_grad_(True)
    assert head_conv_ok(conv, xg)
    y = conv(xg)
    y.backward(gy.to(DEV))
    return y, xg.grad, conv.weight.grad, conv.bias.grad


@pytest.mark.parametrize("n,c,h,w", [(4, 128, 120, 160), (2, 40, 7, 12), (3, 3, 1, 4)])
def test_head_conv_vs_float64(n, c, h, w):
    g = torch.Generator().manual_seed(n + c + h)
    x = torch.rand((n, c, h, w), generator=g) - 0.5
    wt = (torch.rand((1, c, 3, 3), generator=g) - 0.5) * 0.2
    b = torch.rand((1,), generator=g) - 0.5
    gy = torch.rand((n, 1, h, w), generator=g) - 0.5
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, wt, b))
    yr = torch.nn.functional.conv2d(xr, wr, br, 1, 1)
    yr.backward(gy.double())
    y, gx, gw, gb = _run(x, wt, b, gy)
    assert rel_err(y, yr) <= 1e-5, "forward"
    assert rel_err(gx, xr.grad) <= 1e-5, "data gradient"
    assert rel_err(gw, wr.grad) <= 2e-5, "weight gradient"
    assert rel_err(gb, br.grad) <= 1e-5, "bias gradient"
    y2, gx2, gw2, gb2 = _run(x, wt, b, gy)
    assert torch.equal(y, y2) and torch.equal(gx, gx2) and torch.equal(gw, gw2)
    assert torch.equal(gb, gb2)


def test_head_conv_shapes_not_taken():
    from monocular_depth_estimation_amd import _abi
    assert _abi.query("mde_head_conv_supported", 2, 128, 120, 160) == 1
    assert _abi.query("mde_head_conv_supported", 2, 128, 120, 162) == 0  # w % 4
