"""GPU parity of the NewCRF path (HIP/MFMA window attention) vs reference goldens and the oracle.

Tolerances: NewCRF outputs 1e-4 scale-relative, input / parameter gradients
1e-3 (fp32 LayerNorm + GEMM + softmax chains; the reference itself is fp32).
"""
import numpy as np
import pytest
import torch

from oracle import newcrf as onc
from oracle.weights import fill_, seeded
from tests.golden.make_golden import NEWCRF_CASES

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


def close_scaled(a, b, tol, what):
    a = a.detach().double().cpu().numpy() if torch.is_tensor(a) else np.asarray(a, dtype=np.float64)
    b = b.detach().double().cpu().numpy() if torch.is_tensor(b) else np.asarray(b, dtype=np.float64)
    err = float(np.abs(a - b).max())
    assert err <= tol * float(np.abs(b).max()) + 1e-30, f"{what}: {err:.3g} vs {np.abs(b).max():.3g}"


@pytest.mark.parametrize("case", NEWCRF_CASES, ids=[c[0] for c in NEWCRF_CASES])
def test_newcrf_golden(golden, case):
    from monocular_depth_estimation_amd.newcrf_layers import NewCRF
    tag, (ind, emb, vd, heads), _, _ = case
    g = golden("golden_newcrf.npz")
    m = fill_(NewCRF(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads)).to(DEV)
    assert list(m.state_dict().keys()) == list(g[f"{tag}::keys"])
    x = torch.from_numpy(g[f"{tag}::x"]).to(DEV).requires_grad_(True)
    v = torch.from_numpy(g[f"{tag}::v"]).to(DEV).requires_grad_(True)
    y = m(x, v)
    close_scaled(y, g[f"{tag}::y"], 1e-4, "y")
    y.backward(torch.from_numpy(g[f"{tag}::gy"]).to(DEV))
    close_scaled(x.grad, g[f"{tag}::gx"], 1e-3, "gx")
    close_scaled(v.grad, g[f"{tag}::gv"], 1e-3, "gv")
    params = dict(m.named_parameters())
    names = list(g[f"{tag}::grad_names"])
    got = np.array([float(params[n].grad.double().norm()) for n in names])
    np.testing.assert_allclose(got, g[f"{tag}::grad_norms"], rtol=1e-3)
    # full gradients the golden holds (the small parameters: biases, norms, bias tables)
    for key in g:
        if key.startswith(f"{tag}::grad::"):
            n = key[len(f"{tag}::grad::"):]
            close_scaled(params[n].grad, g[key], 1e-3, n)


@pytest.mark.parametrize("b,h,w,emb,heads", [(2, 30, 40, 256, 8), (1, 15, 20, 1024, 32),
                                             (3, 9, 16, 64, 2), (2, 7, 7, 128, 4)])
def test_window_attention_vs_oracle(b, h, w, emb, heads):
    """The attention core alone, both shifts, vs the oracle's pad/roll/partition path."""
    from monocular_depth_estimation_amd.newcrf_layers import window_attention
    torch.manual_seed(0)
    for shift in (0, 3):
        ref = fill_(onc.WindowAttention(emb, 7, heads))
        x = torch.from_numpy(seeded((b, h * w, emb), 5 + shift, -1, 1))
        v = torch.from_numpy(seeded((b, h, w, emb), 6 + shift, -1, 1))
        gy = torch.from_numpy(seeded((b, h * w, emb), 7 + shift, -1, 1))
        # oracle: pad after (here: no) norm, roll, partition, attention (without proj)
        qk_w, qk_b = ref.qk.weight.detach(), ref.qk.bias.detach()
        xg = x.clone().requires_grad_(True)
        vg = v.clone().requires_grad_(True)
        tab = ref.relative_position_bias_table.detach().clone()
        ref.proj = torch.nn.Identity()
        ws = 7
        pb, pr = (ws - h % ws) % ws, (ws - w % ws) % ws
        t = torch.nn.functional.pad(xg.view(b, h, w, emb), (0, 0, 0, pr, 0, pb))
        vv = torch.nn.functional.pad(vg, (0, 0, 0, pr, 0, pb))
        hp, wp = h + pb, w + pr
        mask = onc.shift_mask(hp, wp, ws, 3) if shift else None
        if shift:
            t, vv = torch.roll(t, (-shift, -shift), (1, 2)), torch.roll(vv, (-shift, -shift), (1, 2))
        o = onc.from_windows(ref(onc.to_windows(t, ws), onc.to_windows(vv, ws), mask), ws, hp, wp)
        if shift:
            o = torch.roll(o, (shift, shift), (1, 2))
        o = o[:, :h, :w].reshape(b, h * w, emb)
        o.backward(gy)
        # HIP: qk GEMM on real tokens, the kernel does the rest
        xd = x.to(DEV).requires_grad_(True)
        vd = v.to(DEV).requires_grad_(True)
        wd = qk_w.to(DEV).requires_grad_(True)
        bd = qk_b.to(DEV).requires_grad_(True)
        td = tab.detach().to(DEV).requires_grad_(True)
        od = window_attention(torch.nn.functional.linear(xd, wd, bd), bd, vd, td, h, w, heads, 7, shift)
        close_scaled(od, o, 1e-5, f"out shift={shift}")
        od.backward(gy.to(DEV))
        close_scaled(xd.grad, xg.grad, 1e-4, f"dx shift={shift}")
        close_scaled(vd.grad, vg.grad, 1e-4, f"dv shift={shift}")
        close_scaled(td.grad, ref.relative_position_bias_table.grad, 1e-4, f"dtable shift={shift}")
        gw_ref = ref.qk.weight.grad
        close_scaled(wd.grad, gw_ref, 1e-4, f"dW_qk shift={shift}")
        close_scaled(bd.grad, ref.qk.bias.grad, 1e-4, f"db_qk shift={shift}")


def test_decoder_golden(golden):
    from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import Decoder
    g = golden("golden_newcrf.npz")
    dec = fill_(Decoder()).to(DEV)
    assert list(dec.state_dict().keys()) == list(g["dec::keys"])
    feats = [None] * 18
    for i in (4, 7, 13, 16, 17):
        feats[i] = torch.from_numpy(g[f"dec::feat{i}"]).to(DEV).requires_grad_(True)
    y = dec(feats)
    close_scaled(y, g["dec::y"], 1e-4, "decoder depth")
    y.backward(torch.from_numpy(g["dec::gy"]).to(DEV))
    for i in (4, 7, 13, 16, 17):
        close_scaled(feats[i].grad, g[f"dec::gfeat{i}"], 1e-3, f"gfeat{i}")


@pytest.mark.parametrize("rows,c", [(307200, 128), (1000, 256), (37, 512), (4800, 1024), (1, 128),
                                    (98, 64), (50, 192)])
def test_layernorm_matches_aten(rows, c):
    from monocular_depth_estimation_amd.newcrf_layers import LayerNorm
    ln = LayerNorm(c)
    with torch.no_grad():
        ln.weight.copy_(torch.from_numpy(seeded((c,), 1, 0.5, 1.5)))
        ln.bias.copy_(torch.from_numpy(seeded((c,), 2, -0.5, 0.5)))
    ref = torch.nn.LayerNorm(c).double()
    ref.load_state_dict({k: v.double() for k, v in ln.state_dict().items()})
    x = torch.from_numpy(seeded((rows, c), 3, -2, 3))
    gy = torch.from_numpy(seeded((rows, c), 4, -1, 1))
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy.double())
    ln = ln.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = ln(xd)
    close_scaled(y, yr, 1e-5, "y")
    y.backward(gy.to(DEV))
    close_scaled(xd.grad, xr.grad, 1e-4, "gx")
    close_scaled(ln.weight.grad, ref.weight.grad, 1e-4, "ggamma")
    close_scaled(ln.bias.grad, ref.bias.grad, 1e-4, "gbeta")


@pytest.mark.parametrize("rows,c", [(307200, 128), (37, 512), (4800, 1024), (50, 192)])
def test_add_layernorm_bitwise_vs_separate_add(rows, c):
    """add_layer_norm (one HIP pass: s = x + r and LayerNorm(s); the backward
    adds s's residual gradient in its epilogue) == ATen's add + the HIP
    LayerNorm + autograd's accumulation, bitwise: same fp32 operations."""
    from monocular_depth_estimation_amd import newcrf_layers as nl
    ln = nl.LayerNorm(c).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.from_numpy(seeded((c,), 1, 0.5, 1.5)))
        ln.bias.copy_(torch.from_numpy(seeded((c,), 2, -0.5, 0.5)))
    x0 = torch.from_numpy(seeded((rows, c), 3, -2, 3)).to(DEV)
    r0 = torch.from_numpy(seeded((rows, c), 5, -1, 1)).to(DEV)
    gs = torch.from_numpy(seeded((rows, c), 6, -1, 1)).to(DEV)
    gy = torch.from_numpy(seeded((rows, c), 4, -1, 1)).to(DEV)
    outs = []
    for fused in (True, False):
        old = nl.LN_ADD
        nl.LN_ADD = fused
        try:
            ln.weight.grad = ln.bias.grad = None
            x = x0.clone().requires_grad_(True)
            r = r0.clone().requires_grad_(True)
            s, y = nl.add_layer_norm(x, r, ln)
            torch.autograd.backward([s, y], [gs, gy])
            outs.append((s.detach(), y.detach(), x.grad, r.grad, ln.weight.grad.clone(),
                         ln.bias.grad.clone()))
        finally:
            nl.LN_ADD = old
    for a, b, name in zip(outs[0], outs[1], ("s", "y", "gx", "gr", "ggamma", "gbeta")):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("shape", [(2, 24, 120, 160), (3, 1024, 15, 20), (1, 5, 7, 3), (2, 40, 7, 12),
                                   (1, 72, 9, 20)])
def test_token_transposes_bit_exact(shape):
    from monocular_depth_estimation_amd.newcrf_layers import nchw_to_tokens, tokens_to_nchw
    b, c, h, w = shape
    x = torch.from_numpy(seeded(shape, 9, -1, 1)).to(DEV).requires_grad_(True)
    t = nchw_to_tokens(x)
    assert torch.equal(t, x.flatten(2).transpose(1, 2))
    back = tokens_to_nchw(t, h, w)
    assert torch.equal(back, x)
    g = torch.from_numpy(seeded(shape, 10, -1, 1)).to(DEV)
    back.backward(g)
    assert torch.equal(x.grad, g)


@pytest.mark.parametrize("t,n", [(4800, 512), (307200 // 16, 256), (1000, 4096), (257, 12)])
def test_colsum_and_gelu_bwd_colsum_vs_float64(t, n):
    """The Linear bias gradient (mde_colsum, replacing autograd's grad.sum(0)) and
    the fused GELU backward + fc1 bias gradient (mde_gelu_bwd_colsum; nn.GELU erf
    form, reference newcrf_layers.py:9-27) against float64 torch."""
    from monocular_depth_estimation_amd.newcrf_layers import _LinearGelu, _colsum
    g = torch.Generator().manual_seed(t + n)
    gy = torch.randn((t, n), generator=g)
    assert_close = torch.testing.assert_close
    got = _colsum(gy.to(DEV)).cpu().double()
    ref = gy.double().sum(0)
    assert_close(got, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()) + 1e-4)
    # fused GELU backward through the autograd Function (x @ W1^T + b1 -> gelu)
    k = 8
    x = torch.randn((t, k), generator=g)
    w1 = torch.randn((n, k), generator=g) * 0.5
    b1 = torch.randn((n,), generator=g) * 0.5
    xs = [v.to(DEV).requires_grad_(True) for v in (x, w1, b1)]
    h = _LinearGelu.apply(*xs)
    h.backward(gy.to(DEV))
    xd = [v.double().requires_grad_(True) for v in (x, w1, b1)]
    hd = torch.nn.functional.gelu(torch.nn.functional.linear(*xd))
    hd.backward(gy.double())
    assert_close(h.detach().cpu().double(), hd.detach(), rtol=1e-5, atol=1e-5)
    for a, b in zip(xs, xd):
        assert_close(a.grad.cpu().double(), b.grad, rtol=1e-4,
                     atol=1e-4 * float(b.grad.abs().max()))
