"""mde_linear_wgrad (csrc/mlp.hip): the token-major Linear weight gradient
gw = g^T x (+ gb = column sums of g) of the NewCRF Linears
(src/newcrf_layers.py:9-27,110-149) vs float64 torch, at the cfg4 shapes
(scaled token counts) and odd split remainders; bitwise run to run."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(g, x, bias):
    from monocular_depth_estimation_amd import _abi
    t, m = g.shape
    n = x.shape[1]
    nbytes = _abi.query("mde_linear_wgrad_workspace", t, m, n)
    assert nbytes > 0
    ws = torch.full((nbytes // 4,), float("nan"), device=DEV)
    gw = torch.full((m, n), float("nan"), device=DEV)
    gb = torch.full((m,), float("nan"), device=DEV) if bias else None
    _abi.call("mde_linear_wgrad", _abi.ptr(g), _abi.ptr(x), _abi.ptr(gw),
              _abi.ptr(gb) if bias else None, t, m, n, _abi.ptr(ws), 0, _abi.stream_of(g))
    return gw, gb


@pytest.mark.parametrize("t,m,n,bias", [
    (16 * 120 * 16, 128, 512, True),    # fc2 at 1/4 (tokens scaled down)
    (16 * 120 * 16, 512, 128, False),   # fc1 (the GELU path: no bias here)
    (4800, 1024, 4096, True),           # 1/32 fc2, the full cfg4 token count
    (4800, 4096, 1024, True),
    (16, 128, 128, True),               # one chunk
    (16 * 37, 256, 128, True),          # splits with a ragged last one
    (513 * 16, 384, 256, True)])
def test_linear_wgrad_vs_float64(t, m, n, bias):
    gen = torch.Generator(device=DEV).manual_seed(t + m + n)
    g = torch.randn((t, m), device=DEV, generator=gen)
    x = torch.randn((t, n), device=DEV, generator=gen)
    gw, gb = _run(g, x, bias)
    ref = g.double().t() @ x.double()
    # fp32 MFMA chains of up to a split's tokens (~2400 here) of N(0,1) products:
    # a random walk of roundings of the running sum; the 5-sigma tail over
    # millions of entries measured 6.8e-4 at t = 4800 (sums ~ 70)
    tol = 2e-7 * t + 1e-5
    assert float((gw.double() - ref).abs().max()) <= tol, float((gw.double() - ref).abs().max())
    if bias:
        rb = g.double().sum(0)
        assert float((gb.double() - rb).abs().max()) <= tol
    gw2, gb2 = _run(g, x, bias)
    assert torch.equal(gw, gw2)
    if bias:
        assert torch.equal(gb, gb2)


def test_linear_wgrad_unsupported_shapes():
    from monocular_depth_estimation_amd import _abi
    for t, m, n in ((100, 128, 128), (160, 96, 128), (160, 128, 200), (0, 128, 128)):
        assert _abi.query("mde_linear_wgrad_workspace", t, m, n) == 0


def test_linear_tok_backward_matches_autograd():
    """_LinearTok / _LinearGelu (newcrf_layers.py) with the HIP weight gradient
    vs plain autograd of F.linear (+ GELU) in float64."""
    import torch.nn.functional as F
    from monocular_depth_estimation_amd.newcrf_layers import Mlp
    torch.manual_seed(0)
    mlp = Mlp(128, 512).to(DEV)
    x = torch.randn((2, 40 * 48, 128), device=DEV, requires_grad=True)
    y = mlp(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = x.detach().double().requires_grad_(True)
    w1, b1, w2, b2 = (p.detach().double().requires_grad_(True) for p in
                      (mlp.fc1.weight, mlp.fc1.bias, mlp.fc2.weight, mlp.fc2.bias))
    yd = F.linear(F.gelu(F.linear(xd, w1, b1)), w2, b2)
    yd.backward(gy.double())
    for got, ref in ((x.grad, xd.grad), (mlp.fc1.weight.grad, w1.grad), (mlp.fc1.bias.grad, b1.grad),
                     (mlp.fc2.weight.grad, w2.grad), (mlp.fc2.bias.grad, b2.grad)):
        err = float((got.double() - ref).abs().max())
        assert err <= 1e-4 * max(1.0, float(ref.abs().max())), err


@pytest.mark.parametrize("n,c,h,w", [(16, 128, 120, 160), (3, 1024, 15, 20), (1, 40, 2, 2),
                                     (5, 7, 6, 10)])
def test_chansum_vs_float64(n, c, h, w):
    """mde_chansum (a biased conv's bias gradient, the NewCRF projections'
    `y + bias`, newcrf_layers.py:384-392) vs float64 sums; bitwise run to run."""
    from monocular_depth_estimation_amd import _abi
    g = torch.randn((n, c, h, w), device=DEV, generator=torch.Generator(device=DEV).manual_seed(c))
    nbytes = _abi.query("mde_chansum_workspace", n, c, h * w)
    assert nbytes > 0
    outs = []
    for _ in range(2):
        ws = torch.full((nbytes // 4,), float("nan"), device=DEV)
        gb = torch.full((c,), float("nan"), device=DEV)
        _abi.call("mde_chansum", _abi.ptr(g), _abi.ptr(gb), n, c, h * w, _abi.ptr(ws), 0,
                  _abi.stream_of(g))
        outs.append(gb)
    ref = g.double().sum((0, 2, 3))
    tol = 1e-6 * (n * h * w) ** 0.5 * 4 + 1e-6
    assert float((outs[0].double() - ref).abs().max()) <= tol
    assert torch.equal(outs[0], outs[1])
    assert _abi.query("mde_chansum_workspace", n, c, 6) == 0  # hw % 4 != 0


def test_gemm_table_loads_on_this_image():
    """The shipped TunableOp solution table (gemm_table.py) passes TunableOp's
    validators on this image (PyTorch / HIP / hipBLASLt / rocBLAS / gfx950) and
    a listed shape (cfg4's 1/32-stage fc2, [4800, 4096] x [4096, 1024]^T + b)
    gives the default GEMM's result to fp32 accumulation-order tolerance."""
    import torch.nn.functional as F
    from monocular_depth_estimation_amd import gemm_table
    gen = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn((4800, 4096), device=DEV, generator=gen)
    w = torch.randn((1024, 4096), device=DEV, generator=gen) * 0.02
    b = torch.randn((1024,), device=DEV, generator=gen)
    ref = F.linear(x.double(), w.double(), b.double())
    was = torch.cuda.tunable.is_enabled()
    try:
        assert gemm_table.enable() == gemm_table.TABLE
        y = F.linear(x, w, b)
    finally:
        torch.cuda.tunable.enable(was)
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    assert err <= 1e-5, err
