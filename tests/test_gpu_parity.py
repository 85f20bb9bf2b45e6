"""GPU parity: the HIP path (through the C ABI) vs golden fixtures and the CPU oracle.

Tolerances (written per test): single ops 1e-5 relative (fp32); loss
gradients 1e-4; whole-model depth maps 1e-3 scale-relative (BASELINE.json
north_star); whole-model gradient norms 1e-2 (fp32 conditioning of the
randomly filled net: both the reference and the oracle sit ~2e-3 from a
float64 run, see tests/test_oracle_golden.py).
"""
import numpy as np
import pytest
import torch

from oracle import guidedepth as og
from oracle import ops as oops
from oracle.weights import fill_, seeded
from tests.golden.make_golden import NEAREST_CASES, RESIZE_CASES, VARIANT_BLOCKS

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    import monocular_depth_estimation_amd  # noqa: F401  (loads libmde_hip.so, raises if absent)


def npy(t):
    return t.detach().float().cpu().numpy()


def close(a, b, rtol, atol, what=""):
    np.testing.assert_allclose(npy(a) if torch.is_tensor(a) else a,
                               npy(b) if torch.is_tensor(b) else b, rtol=rtol, atol=atol,
                               err_msg=what)


def close_map(a, b, tol, what=""):
    a = npy(a) if torch.is_tensor(a) else a
    b = npy(b) if torch.is_tensor(b) else b
    err = float(np.abs(a.astype(np.float64) - b).max())
    assert err <= tol * float(np.abs(b).max()) + 1e-30, f"{what}: {err:.3g} vs {np.abs(b).max():.3g}"


def cu(a, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t.requires_grad_(grad)


# ------------------------------------------------------------------ resize
@pytest.mark.parametrize("case", RESIZE_CASES, ids=[c[0] for c in RESIZE_CASES])
def test_bilinear_golden(golden, case):
    from monocular_depth_estimation_amd.functional import bilinear_resize
    name, _, kw = case
    g = golden("golden_resize.npz")
    x = cu(g[f"{name}::x"], True)
    y = bilinear_resize(x, size=kw.get("size"), scale_factor=kw.get("scale_factor"),
                        align_corners=kw.get("align_corners", False))
    close(y, g[f"{name}::y"], 1e-5, 1e-6, name)
    y.backward(cu(g[f"{name}::gy"]))
    close(x.grad, g[f"{name}::gx"], 1e-5, 1e-5, name)


@pytest.mark.parametrize("case", NEAREST_CASES, ids=[c[0] for c in NEAREST_CASES])
def test_nearest_golden_bit_exact(golden, case):
    from monocular_depth_estimation_amd.functional import nearest_resize
    name, _, sf = case
    g = golden("golden_resize.npz")
    x = cu(g[f"{name}::x"], True)
    y = nearest_resize(x, scale_factor=sf)
    close(y, g[f"{name}::y"], 0, 0, name)  # a copy: bit-exact
    y.backward(cu(g[f"{name}::gy"]))
    close(x.grad, g[f"{name}::gx"], 0, 0, name)


@pytest.mark.parametrize("n,c,h,w", [(32, 3, 480, 640), (2, 3, 8, 16), (3, 2, 12, 40),
                                     (2, 3, 10, 20), (1, 1, 6, 12)])
def test_nearest_pyramid_matches_two_nearest_calls(n, c, h, w):
    """GuideDepth.py:46-47's two guides from the fused pass == the two
    nearest_resize calls (x0.5, x0.25) bit-exact; shapes the fused kernel does
    not take (h % 4, w % 8) and inputs that need a gradient fall back to them."""
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.functional import nearest_pyramid, nearest_resize
    x = torch.rand((n, c, h, w), device=DEV)
    fused = bool(_abi.query("mde_nearest_pyramid_supported", n, c, h, w))
    assert fused == (h % 4 == 0 and w % 8 == 0)
    half, quarter = nearest_pyramid(x)
    assert torch.equal(half, nearest_resize(x, scale_factor=0.5))
    assert torch.equal(quarter, nearest_resize(x, scale_factor=0.25))
    assert torch.equal(half, x[:, :, ::2, ::2][:, :, :h // 2, :w // 2])
    xg = x.clone().requires_grad_(True)
    hg, qg = nearest_pyramid(xg)
    assert hg.requires_grad and qg.requires_grad
    (hg.sum() + 2 * qg.sum()).backward()
    ref = torch.zeros_like(x)
    ref[:, :, ::2, ::2][:, :, :h // 2, :w // 2] += 1
    ref[:, :, ::4, ::4][:, :, :h // 4, :w // 4] += 2
    assert torch.equal(xg.grad, ref)


@pytest.mark.parametrize("shape,kw", [
    ((32, 16, 240, 320), dict(scale_factor=2)),           # up_3 input, BASELINE cfg2
    ((3, 5, 3, 6), dict(scale_factor=2)),                 # x2, column pairs, short planes
    ((2, 4, 9, 130), dict(scale_factor=2)),               # x2, pairs across two blocks
    ((2, 3, 11, 7), dict(scale_factor=2)),                # x2, odd width: per-column kernel
    ((32, 64, 8, 10), dict(size=(60, 80))),               # DDRNet spp -> H/8 (x7.5)
    ((32, 64, 15, 20), dict(size=(60, 80))),              # compression4 (x4)
    ((16, 1, 120, 160), dict(scale_factor=4)),            # NewCRF head x4 (cfg4)
    ((2, 64, 2, 3), dict(size=(8, 12))),                  # DDRNet compression4 at 64x96 (x4 by size)
    ((4, 64, 15, 20), dict(size=(60, 80))),               # DDRNet compression4 at 640x480 (x4 by size)
    ((2, 3, 9, 70), dict(scale_factor=4)),                # x4, odd rows, two column blocks
    ((1, 2, 5, 3), dict(scale_factor=4)),                 # x4, tiny plane (every edge case)
    ((2, 2, 7, 66), dict(scale_factor=8)),                # x8
    ((2, 3, 100, 150), dict(size=(310, 470))),            # plane > LDS: banded kernel
    ((1, 2, 10, 10), dict(size=(200, 210))),              # x20: per-pixel gather kernel
    ((2, 3, 37, 41), dict(size=(111, 90), align_corners=True)),
])
def test_bilinear_full_size_adjoint_and_oracle_rows(shape, kw):
    """At cfg2 sizes: <fwd(x), g> == <x, bwd(g)> (adjointness), plus oracle parity on 2 samples."""
    from monocular_depth_estimation_amd.functional import bilinear_resize
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand(shape, device=DEV, generator=gen).requires_grad_(True)
    y = bilinear_resize(x, **kw)
    gy = torch.rand(y.shape, device=DEV, generator=gen) - 0.5
    y.backward(gy)
    lhs = (y.double() * gy.double()).sum()
    rhs = (x.double() * x.grad.double()).sum()
    assert abs(float(lhs - rhs)) <= 1e-5 * float(y.double().abs().sum())
    xs = x.detach()[:2].cpu().requires_grad_(True)
    ys = oops.bilinear(xs, **kw)
    # The source coordinate s = scale*(dst+0.5)-0.5 carries one fp32 ulp of
    # slack (7.6e-6 once s >= 64: FMA-contracted or not, per compiler), which
    # moves the interpolation weight by that much: atol scales with it.
    ulp = float(np.spacing(np.float32(max(shape[-2:]))))
    close(y[:2], ys, 1e-5, max(1e-6, 2 * ulp), "fwd vs oracle")
    ys.backward(gy[:2].cpu())
    close(x.grad[:2], xs.grad, 1e-5, max(1e-5, 8 * ulp), "bwd vs oracle")


# --------------------------------------------------------------------- SE
@pytest.mark.parametrize("tag,ch,red", [("se16", 16, 1), ("se32r4", 32, 4)])
def test_se_golden(golden, tag, ch, red):
    from monocular_depth_estimation_amd.GuideDepth.model.modules import SELayer
    g = golden("golden_blocks.npz")
    m = fill_(SELayer(ch, reduction=red)).to(DEV)
    x = cu(g[f"{tag}::x"], True)
    y = m(x)
    close(y, g[f"{tag}::y"], 1e-5, 1e-6)
    y.backward(cu(g[f"{tag}::gy"]))
    close(x.grad, g[f"{tag}::gx"], 1e-5, 1e-6)
    close(m.fc[0].weight.grad, g[f"{tag}::gw1"], 1e-4, 1e-5)
    close(m.fc[2].weight.grad, g[f"{tag}::gw2"], 1e-4, 1e-5)


@pytest.mark.parametrize("n,ca,cb,h,w", [(2, 8, 8, 30, 41), (4, 32, 32, 120, 160), (32, 8, 8, 480, 640)])
def test_se_cat_vs_oracle(n, ca, cb, h, w):
    from monocular_depth_estimation_amd.functional import se_cat
    c = ca + cb
    xa = torch.from_numpy(seeded((n, ca, h, w), 1, -1, 1))
    xb = torch.from_numpy(seeded((n, cb, h, w), 2, -1, 1))
    w1 = torch.from_numpy(seeded((c, c), 3, -0.3, 0.3))
    w2 = torch.from_numpy(seeded((c, c), 4, -0.3, 0.3))
    gy = torch.from_numpy(seeded((n, c, h, w), 5, -1, 1))
    ins = [t.to(DEV).requires_grad_(True) for t in (xa, xb, w1, w2)]
    y = se_cat(*ins)
    y.backward(gy.to(DEV))
    k = min(n, 2)  # oracle on the first samples (per-sample op), weight grads on all
    refs = [t[:k].clone().requires_grad_(True) if i < 2 else t.clone().requires_grad_(True)
            for i, t in enumerate((xa, xb, w1, w2))]
    yr = oops.se(torch.cat(refs[:2], 1), refs[2], refs[3])
    close(y[:k], yr, 1e-5, 1e-6, "fwd")
    yr.backward(gy[:k])
    close(ins[0].grad[:k], refs[0].grad, 1e-4, 1e-6, "gxa")
    close(ins[1].grad[:k], refs[1].grad, 1e-4, 1e-6, "gxb")
    if k == n:
        close(ins[2].grad, refs[2].grad, 1e-4, 1e-4, "gw1")
        close(ins[3].grad, refs[3].grad, 1e-4, 1e-4, "gw2")


# ------------------------------------------------------------ skip fusion
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 32, 12, 16), (2, 32, 16, 24, 32),
                                            (2, 16, 1, 48, 64), (2, 8, 4, 9, 11),
                                            (2, 40, 24, 7, 13), (32, 16, 1, 480, 640),
                                            (4, 64, 32, 120, 160), (2, 32, 16, 240, 320),
                                            (2, 64, 32, 10, 10)])
def test_skip_reduce_vs_oracle(n, cin, cout, h, w):
    from monocular_depth_estimation_amd.functional import skip_reduce
    r = torch.from_numpy(seeded((n, cin, h, w), 11, -1, 1))
    d = torch.from_numpy(seeded((n, cin, h, w), 12, -1, 1))
    wt = torch.from_numpy(seeded((cout, cin, 1, 1), 13, -0.5, 0.5))
    b = torch.from_numpy(seeded((cout,), 14, -0.5, 0.5))
    gy = torch.from_numpy(seeded((n, cout, h, w), 15, -1, 1))
    ins = [t.to(DEV).requires_grad_(True) for t in (r, d, wt, b)]
    y = skip_reduce(*ins)
    y.backward(gy.to(DEV))
    refs = [t.clone().double().requires_grad_(True) for t in (r, d, wt, b)]
    yr = oops.skip_reduce(*refs)
    close(y, yr, 1e-5, 1e-5, "fwd")
    yr.backward(gy.double())
    close(ins[0].grad, refs[0].grad, 1e-5, 1e-5, "g residual")
    close(ins[1].grad, refs[1].grad, 1e-5, 1e-5, "g depth")
    scale = float(refs[2].grad.abs().max())
    close(ins[2].grad, refs[2].grad, 1e-4, 1e-5 * scale, "g weight")
    close(ins[3].grad, refs[3].grad, 1e-4, 1e-5 * float(refs[3].grad.abs().max()), "g bias")


# ------------------------------------------------------------------ losses
@pytest.mark.parametrize("tag", ["rand", "close", "anti"])
def test_ssim_golden(golden, tag):
    from monocular_depth_estimation_amd.loss import SSIM
    g = golden("golden_losses.npz")
    x = cu(g[f"ssim_{tag}::x"], True)
    y = cu(g[f"ssim_{tag}::y"], True)
    v = SSIM()(x, y)
    close(v, g[f"ssim_{tag}::loss"], 1e-5, 1e-7)
    v.backward()
    # elementwise 1e-4 relative, with an absolute floor of 1e-4 * max|grad|
    # for entries that are themselves rounding-level (cancellation in S)
    for got, key in ((x.grad, "gx"), (y.grad, "gy")):
        ref = g[f"ssim_{tag}::{key}"]
        close(got, ref, 1e-4, 1e-4 * float(np.abs(ref).max()), key)


def test_train_objective_golden(golden):
    """DepthNorm fused into the SSIM+L1 kernel == the reference's three calls."""
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.utils import DepthNorm
    g = golden("golden_losses.npz")
    pred = cu(g["train::pred"], True)
    depth = cu(g["train::depth"])
    close(DepthNorm(depth), g["train::depth_n"], 1e-6, 1e-7)
    crit = SSIML1(1.0, 0.1, depth_norm=True)
    loss = crit(pred, depth)
    close(loss, g["train::loss"], 1e-5, 1e-7)
    close(crit.last_parts[1], g["train::ssim"], 1e-5, 1e-7)
    close(crit.last_parts[2], g["train::l1"], 1e-5, 1e-7)
    (2.0 * loss).backward()
    ref = 2.0 * g["train::gpred"]
    close(pred.grad, ref, 1e-4, 1e-4 * float(np.abs(ref).max()))


def test_silog_golden(golden):
    """Silog_loss_variance (loss.py:116-129) on the device vs the reference's value
    (golden train::silog: prediction vs the DepthNorm'd target)."""
    from monocular_depth_estimation_amd.loss import Silog_loss_variance
    g = golden("golden_losses.npz")
    pred = cu(g["train::pred"], True)
    dn = cu(g["train::depth_n"])
    val = Silog_loss_variance()(pred, dn)
    close(val, g["train::silog"], 1e-5, 1e-7)
    val.backward()  # the reference's value is differentiable too: finite gradient
    assert torch.isfinite(pred.grad).all()
    # against the oracle's boolean-mask form, incl. a target with invalid pixels and p <= 1e-6
    p = torch.from_numpy(seeded((2, 1, 48, 64), 31, -0.1, 2.0))
    t = torch.from_numpy(seeded((2, 1, 48, 64), 32, -0.2, 3.0))
    close(Silog_loss_variance(0.85)(p.to(DEV), t.to(DEV)), oops.silog(p, t), 1e-5, 1e-6)
    close(Silog_loss_variance(0.5)(p.to(DEV), t.to(DEV)), oops.silog(p, t, 0.5), 1e-5, 1e-6)


@pytest.mark.parametrize("shape", [(1, 1, 2, 2), (1, 2, 5, 7), (3, 1, 17, 70), (2, 1, 50, 260),
                                   (2, 1, 36, 132), (32, 1, 480, 640), (1, 1, 3, 3), (1, 1, 2, 121),
                                   (2, 1, 130, 61), (1, 1, 97, 2), (4, 1, 64, 120)])
def test_ssim_l1_vs_oracle_sizes(shape):
    """Strip (60 columns) / row-chunk boundaries, 2- and 3-wide images (both
    reflections on one pixel), the full cfg2 batch."""
    from monocular_depth_estimation_amd.functional import minmax, ssim3_l1
    p = torch.from_numpy(seeded(shape, 21, 0, 1))
    d = torch.from_numpy(seeded(shape, 22, 0.1, 10.0))
    pg = p.to(DEV).requires_grad_(True)
    loss, parts = ssim3_l1(pg, d.to(DEV), 1.0, 0.1, target_minmax=minmax(d.to(DEV)))
    loss.backward()
    pr = p.clone().double().requires_grad_(True)
    ref = oops.train_loss(pr, d.double())
    ref.backward()
    close(loss, ref, 2e-5, 1e-7, "loss")
    scale = float(pr.grad.abs().max())
    close(pg.grad, pr.grad, 1e-3, 1e-4 * scale, "grad")


def test_ssim_identical_inputs_full_size():
    """SSIM(x, x) = 0 everywhere with (1-S)/2 = 0 on the clamp edge; L1 = 0, grad = 0."""
    from monocular_depth_estimation_amd.functional import ssim3_l1
    x = torch.rand((32, 1, 480, 640), device=DEV).requires_grad_(True)
    loss, parts = ssim3_l1(x, x.detach(), 1.0, 0.1)
    loss.backward()
    assert abs(float(parts[1])) < 1e-6 and float(parts[2]) == 0.0
    assert float(x.grad.abs().max()) < 1e-6


@pytest.mark.parametrize("tag", ["dl_alh", "dl_mask", "dl_small", "dl_ssim_only"])
def test_depth_loss_golden(golden, tag):
    from monocular_depth_estimation_amd.GuideDepth.losses import Depth_Loss
    g = golden("golden_losses.npz")
    a, b, gm, mx = (float(v) for v in g[f"{tag}::params"])
    x = cu(g[f"{tag}::pred"], True)
    v = Depth_Loss(a, b, gm, maxDepth=mx)(x, cu(g[f"{tag}::gt"]))
    close(v, g[f"{tag}::loss"], 1e-5, 1e-7)
    (3.0 * v).backward()
    ref = 3.0 * g[f"{tag}::gpred"]
    close(x.grad, ref, 1e-4, 1e-4 * float(np.abs(ref).max()))


@pytest.mark.parametrize("shape,params", [
    ((2, 1, 100, 130), (0.1, 1.0, 1.0, 10.0)),   # 3 column strips (54 wide), 4 row chunks
    ((1, 2, 11, 11), (0.1, 1.0, 1.0, 10.0)),     # smallest full window, one strip
    ((3, 1, 45, 55), (0.0, 1.0, 0.0, 1.0)),      # SSIM only: 55 = one strip + 1 column
    ((2, 1, 70, 108), (0.5, 0.0, 1.0, 10.0)),    # no SSIM: L1 + gradient only
    ((2, 1, 64, 97), (1.0, 0.0, 0.0, 10.0)),     # masked L1 (odd numel tail)
])
def test_depth_loss_streaming_shapes_vs_oracle(shape, params):
    """The register-streaming Depth_Loss kernels (strip / chunk borders, the
    zero padding of the 11x11 window at every image edge, each mode) against
    the float64 oracle: loss 1e-5, gradient 1e-4 of its scale."""
    from monocular_depth_estimation_amd.functional import depth_loss
    a, b, gm, mx = params
    p = torch.from_numpy(seeded(shape, 41, 0, mx))
    t = torch.from_numpy(seeded(shape, 42, 0, mx))
    if b == 0.0 and gm == 0.0:
        t[..., ::3, ::2] = 0.0  # invalid pixels of the masked mode
    pg = p.to(DEV).requires_grad_(True)
    loss, _ = depth_loss(pg, t.to(DEV), a, b, gm, mx)
    (2.0 * loss).backward()
    pr = p.clone().double().requires_grad_(True)
    ref = oops.depth_loss(pr, t.double(), a, b, gm, mx)
    (2.0 * ref).backward()
    close(loss, ref, 1e-5, 1e-7)
    close(pg.grad, pr.grad, 1e-4, 1e-4 * float(pr.grad.abs().max()))


def test_depth_loss_full_size_vs_oracle_crop():
    """cfg2-sized Depth_Loss runs; a 2-sample crop matches the oracle."""
    from monocular_depth_estimation_amd.functional import depth_loss
    p = torch.from_numpy(seeded((4, 1, 96, 128), 31, 0, 10))
    t = torch.from_numpy(seeded((4, 1, 96, 128), 32, 0, 10))
    pg = p.to(DEV).requires_grad_(True)
    loss, _ = depth_loss(pg, t.to(DEV), 0.1, 1.0, 1.0, 10.0)
    loss.backward()
    pr = p.clone().double().requires_grad_(True)
    ref = oops.depth_loss(pr, t.double(), 0.1, 1.0, 1.0, 10.0)
    ref.backward()
    close(loss, ref, 1e-5, 1e-7)
    close(pg.grad, pr.grad, 1e-3, 1e-4 * float(pr.grad.abs().max()))
    big = torch.rand((32, 1, 480, 640), device=DEV).requires_grad_(True)
    v, parts = depth_loss(big, torch.rand((32, 1, 480, 640), device=DEV), 0.1, 1.0, 1.0, 10.0)
    v.backward()
    assert torch.isfinite(big.grad).all() and torch.isfinite(v)


# ------------------------------------------------------------- the model
@pytest.mark.parametrize("tag,cfg", [("gub1", (64, 64, 32)), ("gub2", (32, 32, 16)),
                                     ("gub3", (16, 16, 1))])
def test_guided_block_golden(golden, tag, cfg):
    from monocular_depth_estimation_amd.GuideDepth.model.modules import Guided_Upsampling_Block
    g = golden("golden_blocks.npz")
    m = fill_(Guided_Upsampling_Block(*cfg)).to(DEV).train()
    guide = cu(g[f"{tag}::guide"], True)
    depth = cu(g[f"{tag}::depth"], True)
    y = m(guide, depth)
    close_map(y, g[f"{tag}::y"], 1e-4, "y")
    y.backward(cu(g[f"{tag}::gy"]))
    close_map(depth.grad, g[f"{tag}::gdepth"], 1e-4, "gdepth")
    close_map(guide.grad, g[f"{tag}::gguide"], 1e-4, "gguide")


@pytest.mark.parametrize("tag", sorted(VARIANT_BLOCKS))
def test_guided_block_variants_golden(golden, tag):
    """Reference API variants: guidance_type 'raw' (guide concatenated raw) /
    other (no guide), channel_attention=False (modules.py:62-65,80,91-96) --
    the unfused paths of the block -- against the reference's own outputs and
    every parameter gradient (1e-4 scale-relative)."""
    from monocular_depth_estimation_amd.GuideDepth.model.modules import Guided_Upsampling_Block
    g = golden("golden_variants.npz")
    cin, e, cout, ca, gt = VARIANT_BLOCKS[tag]
    m = fill_(Guided_Upsampling_Block(cin, e, cout, channel_attention=ca,
                                      guidance_type=gt)).to(DEV).train()
    guide = cu(g[f"{tag}::guide"], True)
    depth = cu(g[f"{tag}::depth"], True)
    y = m(guide, depth)
    close_map(y, g[f"{tag}::y"], 1e-4, "y")
    y.backward(cu(g[f"{tag}::gy"]))
    close_map(depth.grad, g[f"{tag}::gdepth"], 1e-4, "gdepth")
    if f"{tag}::gguide" in g:
        close_map(guide.grad, g[f"{tag}::gguide"], 1e-4, "gguide")
    else:
        assert guide.grad is None
    params = dict(m.named_parameters())
    names = list(g[f"{tag}::grad_names"])
    norms = g[f"{tag}::grad_norms"]
    for n, ref in zip(names, norms):
        if n.endswith(("_conv.0.bias", "_conv.3.bias")) or ref < 1e-6 * norms.max():
            continue  # conv biases feeding train-mode BN: true gradient 0 (noise only)
        got = float(params[n].grad.double().norm())
        assert abs(got - ref) <= 1e-4 * ref + 1e-7 * norms.max(), (n, got, ref)
        if f"{tag}::grad::{n}" in g:
            close_map(params[n].grad, g[f"{tag}::grad::{n}"], 1e-4, n)


def test_guidedepth_s_golden(golden):
    """GuideDepth-S (loader.py:18-19: up / inner features [32, 8, 4]) at
    128x192: depth maps (train and eval BN) 1e-3, loss 1e-4, gradient norms
    vs the float64 oracle (2e-2 max / 5e-3 median, see _grad_norm_check)."""
    from monocular_depth_estimation_amd.GuideDepth.model.loader import model_builder
    from monocular_depth_estimation_amd.loss import SSIML1
    g = golden("golden_variants.npz")
    model = fill_(model_builder("GuideDepth-S", pretrained=False)).to(DEV).train()
    assert list(model.state_dict().keys()) == list(g["gds::state_dict_keys"])
    x = cu(g["gds::x"])
    pred = model(x)
    close_map(pred, g["gds::train_pred"], 1e-3, "train-mode depth map")
    loss = SSIML1(1.0, 0.1)(pred, cu(g["gds::depth"]))
    close(loss, g["gds::train_loss"], 1e-4, 1e-7)
    loss.backward()
    _grad_norm_check(model, g, g["gds::x"], g["gds::depth"], prefix="gds::",
                     features=((32, 8, 4), (32, 8, 4)))
    model.eval()
    with torch.no_grad():
        close_map(model(x), g["gds::eval_pred"], 1e-3, "eval-mode depth map")


def _grad_norm_check(model, g, x, depth, prefix="", features=None):
    """Per-parameter grad norms vs a FLOAT64 run of the oracle (the truth).

    The fp32 reference itself sits at max 5.8e-3 / median 1.7e-3 relative
    from that truth on this randomly filled net (measured on the golden);
    the HIP path must stay within 2e-2 max / 5e-3 median.  The max is one
    ill-conditioned parameter: layer5's BatchNorms normalise 2 x 1 x 2 = 4
    values at 64x96, and the convolutions still on MIOpen there (the 1/64
    planes) take whichever solver MIOpen picks from its on-disk databases,
    which earlier processes on the box write: layer5.0.bn3.weight measured
    5.3e-3 in a box's first process and 1.1e-2 in its second with the HIP
    kernels unchanged, 1.5e-2 inside the full suite (gpurun_out/r06ah,
    r06full4; tools/gd_grad_probe.py).
    """
    names = list(g[f"{prefix}grad_names"])
    ref32 = g[f"{prefix}grad_norms"]
    kw = {} if features is None else dict(up_features=features[0], inner_features=features[1])
    truth = fill_(og.GuideDepth(**kw)).double().train()
    oops.train_loss(truth(torch.from_numpy(x).double()), torch.from_numpy(depth).double()).backward()
    tp = dict(truth.named_parameters())
    t64 = np.array([float(tp[n].grad.norm()) for n in names])
    params = dict(model.named_parameters())
    got = np.array([float(params[n].grad.double().norm()) for n in names])
    keep = ref32 > 1e-7 * ref32.max()
    keep &= np.array(["bias" not in n or not any(k in n for k in ("conv1.0", "conv1.3", "_conv.0", "_conv.3"))
                      for n in names])
    rel = np.abs(got - t64)[keep] / t64[keep]
    worst = sorted(zip(rel, np.array(names)[keep]), reverse=True)[:5]
    assert rel.max() <= 2e-2 and np.median(rel) <= 5e-3, f"worst {worst}, median {np.median(rel):.2e}"


def test_guidedepth_golden(golden):
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    g = golden("golden_guidedepth.npz")
    model = fill_(GuideDepth(pretrained=False)).to(DEV).train()
    x = cu(g["x"])
    pred = model(x)
    close_map(pred, g["train_pred"], 1e-3, "train-mode depth map")
    loss = SSIML1(1.0, 0.1)(pred, cu(g["depth"]))
    close(loss, g["train_loss"], 1e-4, 1e-7)
    loss.backward()
    _grad_norm_check(model, g, g["x"], g["depth"])
    model.eval()
    with torch.no_grad():
        close_map(model(x), g["eval_pred"], 1e-3, "eval-mode depth map")


def test_train_sequence_golden(golden):
    """Loss-curve parity: 5 steps of the train.py recipe (eval switch after step 0)."""
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import Trainer, World, make_adam
    g = golden("golden_trainseq.npz")
    model = fill_(GuideDepth(pretrained=False)).to(DEV)
    trainer = Trainer(model, make_adam(model, 1e-4), SSIML1(1.0, 0.1), World(device=torch.device(DEV)))
    trainer.begin_epoch()
    losses = []
    for k in range(len(g["losses"])):
        image = cu(seeded((2, 3, 64, 96), 100 + k, 0, 1))
        depth = cu(seeded((2, 1, 64, 96), 200 + k, 0.1, 10.0))
        losses.append(float(trainer.step(image, depth)))
        trainer.after_step(k)
    # Step 0 to 1e-5.  Later steps: Adam's first update moves every conv bias in
    # front of a BatchNorm by ~lr * sign(g) where the true gradient is 0 (its sign
    # is rounding noise), and from step 1 BN runs in eval mode where those biases
    # matter; the reference's own ATen ops (the oracle) span up to 6.0e-3 from
    # this golden when only the CPU thread count changes (1/2/3/8 threads:
    # 6.0e-3 / 4.7e-3 / 2.5e-3 / 2.7e-3), so the curve is held to 1e-2.
    np.testing.assert_allclose(losses[0], g["losses"][0], rtol=1e-5)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-2)


def test_train_sequence_golden_graph(golden):
    """The same loss-curve golden through GraphTrainer (the path bench.py and
    `train.py --graph` replay): step 0 in train mode, the eval-mode switch
    after it (src/train.py:79,134-136,161), steps 1.. from the captured
    eval-mode graph (one eager warm-up step; test_gpu_graph.py's two-epoch test
    covers a captured train-mode step next to it).  Tolerances as the eager
    Trainer's (step 0 1e-5, curve 1e-2)."""
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, World
    g = golden("golden_trainseq.npz")
    model = fill_(GuideDepth(pretrained=False)).to(DEV)
    trainer = GraphTrainer(model, SSIML1(1.0, 0.1), World(device=torch.device(DEV)), lr=1e-4,
                           eager_steps=1, eval_quirk=True)
    trainer.begin_epoch()
    losses = []
    try:
        for k in range(len(g["losses"])):
            image = cu(seeded((2, 3, 64, 96), 100 + k, 0, 1))
            depth = cu(seeded((2, 1, 64, 96), 200 + k, 0.1, 10.0))
            losses.append(float(trainer.step(image, depth)))
            trainer.after_step(k)
        assert sorted(trainer.graphs) == ["eval"]
    finally:
        trainer.close()
    np.testing.assert_allclose(losses[0], g["losses"][0], rtol=1e-5)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-2)


def test_guidedepth_cfg2_shape_runs_and_matches_oracle_encoder_free_parts():
    """640x480 bs=2 forward+backward on the HIP path vs the CPU oracle (1e-3 map tolerance)."""
    from monocular_depth_estimation_amd import GuideDepth
    model = fill_(GuideDepth(pretrained=False)).to(DEV).train()
    ref = fill_(og.GuideDepth()).train()
    x = torch.from_numpy(seeded((2, 3, 480, 640), 71, 0, 1))
    pred = model(x.to(DEV))
    with torch.no_grad():
        rp = ref(x)
    close_map(pred, rp, 1e-3, "640x480 depth map")


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 16, 8, 48, 64), (3, 16, 16, 8, 8), (2, 32, 16, 24, 32),
                                            (2, 32, 32, 16, 16), (2, 64, 32, 12, 16),
                                            (1, 32, 64, 8, 8), (2, 16, 32, 8, 16), (2, 64, 64, 12, 16),
                                            (32, 16, 8, 480, 640)])
def test_pointwise_conv_vs_aten(n, cin, cout, h, w):
    """HIP MFMA 1x1 convolution (the BN-folded guided-upsampling convs) vs ATen float64."""
    from monocular_depth_estimation_amd.nn import _Pointwise
    x = torch.from_numpy(seeded((n, cin, h, w), 21, -1, 1))
    wt = torch.from_numpy(seeded((cout, cin, 1, 1), 22, -0.5, 0.5))
    gy = torch.from_numpy(seeded((n, cout, h, w), 23, -1, 1))
    xd, wd = x.to(DEV).requires_grad_(True), wt.to(DEV).requires_grad_(True)
    y = _Pointwise.apply(xd, wd)
    y.backward(gy.to(DEV))
    xr, wr = x.double().requires_grad_(True), wt.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr)
    yr.backward(gy.double())
    close(y, yr, 1e-5, 1e-5, "fwd")
    close(xd.grad, xr.grad, 1e-5, 1e-5, "gx")
    close(wd.grad, wr.grad, 1e-4, 1e-5 * float(wr.grad.abs().max()), "gw")
