"""Pins the CPU oracle (oracle/) to golden vectors captured from the reference.

Fixtures: tests/golden/*.npz, written by tests/golden/make_golden.py which
imports /root/reference/src.  CPU only.
"""
import numpy as np
import pytest
import torch

from oracle import ops
from oracle import guidedepth as og
from oracle.weights import fill_, seeded

from tests.golden.make_golden import NEAREST_CASES, RESIZE_CASES, VARIANT_BLOCKS

torch.set_num_threads(4)


def close(a, b, rtol=1e-5, atol=1e-6, what=""):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


def close_map(a, b, tol, what=""):
    """Depth-map parity: max |a - b| <= tol * max |b| (scale-relative)."""
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    err = float(np.abs(a.astype(np.float64) - b).max())
    assert err <= tol * float(np.abs(b).max()), f"{what}: max err {err:.3g} vs scale {np.abs(b).max():.3g}"


@pytest.mark.parametrize("case", RESIZE_CASES, ids=[c[0] for c in RESIZE_CASES])
def test_bilinear_matches_reference(golden, case):
    name, _, kw = case
    g = golden("golden_resize.npz")
    x = torch.from_numpy(g[f"{name}::x"]).requires_grad_(True)
    y = ops.bilinear(x, **kw)
    close(y, g[f"{name}::y"], what=name)
    y.backward(torch.from_numpy(g[f"{name}::gy"]))
    close(x.grad, g[f"{name}::gx"], rtol=1e-5, atol=1e-5, what=name)


@pytest.mark.parametrize("case", NEAREST_CASES, ids=[c[0] for c in NEAREST_CASES])
def test_nearest_matches_reference(golden, case):
    name, _, sf = case
    g = golden("golden_resize.npz")
    x = torch.from_numpy(g[f"{name}::x"]).requires_grad_(True)
    y = ops.nearest(x, scale_factor=sf)
    close(y, g[f"{name}::y"], rtol=0, atol=0, what=name)
    y.backward(torch.from_numpy(g[f"{name}::gy"]))
    close(x.grad, g[f"{name}::gx"], rtol=0, atol=0, what=name)


@pytest.mark.parametrize("tag,ch,red", [("se16", 16, 1), ("se32r4", 32, 4)])
def test_se_matches_reference(golden, tag, ch, red):
    g = golden("golden_blocks.npz")
    m = fill_(og.SELayer(ch, reduction=red))
    x = torch.from_numpy(g[f"{tag}::x"]).requires_grad_(True)
    y = m(x)
    close(y, g[f"{tag}::y"])
    y.backward(torch.from_numpy(g[f"{tag}::gy"]))
    close(x.grad, g[f"{tag}::gx"], atol=1e-6)
    close(m.fc[0].weight.grad, g[f"{tag}::gw1"], atol=1e-5)
    close(m.fc[2].weight.grad, g[f"{tag}::gw2"], atol=1e-5)


def null_grad_params(module):
    """Biases of convs feeding a train-mode BatchNorm: their true gradient is 0,
    so both sides hold only rounding noise there (not comparable)."""
    out = set()
    for name, m in module.named_modules():
        if isinstance(m, torch.nn.Sequential):
            kids = list(m.children())
            for i in range(len(kids) - 1):
                if isinstance(kids[i], torch.nn.Conv2d) and kids[i].bias is not None and \
                        isinstance(kids[i + 1], torch.nn.BatchNorm2d):
                    out.add(f"{name}.{i}.bias" if name else f"{i}.bias")
    return out


def _check_grad_summary(module, g, prefix, rtol=1e-4):
    names = list(g[f"{prefix}grad_names"])
    params = dict(module.named_parameters())
    assert sorted(names) == sorted(n for n, p in params.items() if p.grad is not None)
    skip = null_grad_params(module)
    ref_norms = g[f"{prefix}grad_norms"]
    # any other parameter whose true gradient is 0 (e.g. a BN bias feeding only
    # train-mode BNs) shows up as a norm ~1e-10 of the largest: noise only
    skip |= {n for n, v in zip(names, ref_norms) if v < 1e-7 * ref_norms.max()}
    keep = [i for i, n in enumerate(names) if n not in skip]
    assert len(keep) > 0.5 * len(names)
    got_norm = np.array([float(params[names[i]].grad.double().norm()) for i in keep])
    np.testing.assert_allclose(got_norm, g[f"{prefix}grad_norms"][keep], rtol=rtol, atol=1e-7)
    for n in names:
        if n in skip:
            continue
        key = f"{prefix}grad::{n}"
        if key in g:
            ref = g[key]
            scale = max(np.abs(ref).max(), 1e-6)
            close(params[n].grad, ref, rtol=rtol, atol=rtol * scale, what=n)


@pytest.mark.parametrize("tag,cfg", [("gub1", (64, 64, 32)), ("gub2", (32, 32, 16)),
                                     ("gub3", (16, 16, 1))])
def test_guided_block_matches_reference(golden, tag, cfg):
    g = golden("golden_blocks.npz")
    m = fill_(og.GuidedUpsamplingBlock(*cfg)).train()
    guide = torch.from_numpy(g[f"{tag}::guide"]).requires_grad_(True)
    depth = torch.from_numpy(g[f"{tag}::depth"]).requires_grad_(True)
    y = m(guide, depth)
    close(y, g[f"{tag}::y"], rtol=1e-4, atol=1e-5)
    y.backward(torch.from_numpy(g[f"{tag}::gy"]))
    close(depth.grad, g[f"{tag}::gdepth"], rtol=1e-4, atol=1e-5)
    close(guide.grad, g[f"{tag}::gguide"], rtol=1e-4, atol=1e-5)
    _check_grad_summary(m, g, f"{tag}::")


@pytest.mark.parametrize("tag", sorted(VARIANT_BLOCKS))
def test_guided_block_variants_match_reference(golden, tag):
    """guidance_type 'raw' / other and channel_attention=False (modules.py:62-65,80,91-96)."""
    g = golden("golden_variants.npz")
    cin, e, cout, ca, gt = VARIANT_BLOCKS[tag]
    m = fill_(og.GuidedUpsamplingBlock(cin, e, cout, channel_attention=ca,
                                        guidance_type=gt)).train()
    guide = torch.from_numpy(g[f"{tag}::guide"]).requires_grad_(True)
    depth = torch.from_numpy(g[f"{tag}::depth"]).requires_grad_(True)
    y = m(guide, depth)
    close(y, g[f"{tag}::y"], rtol=1e-4, atol=1e-5)
    y.backward(torch.from_numpy(g[f"{tag}::gy"]))
    close(depth.grad, g[f"{tag}::gdepth"], rtol=1e-4, atol=1e-5)
    if f"{tag}::gguide" in g:
        close(guide.grad, g[f"{tag}::gguide"], rtol=1e-4, atol=1e-5)
    else:
        assert guide.grad is None
    _check_grad_summary(m, g, f"{tag}::")


def test_guidedepth_s_matches_reference(golden):
    """GuideDepth-S = GuideDepth(up/inner features [32, 8, 4]) (loader.py:18-19)."""
    g = golden("golden_variants.npz")
    model = fill_(og.GuideDepth(up_features=(32, 8, 4), inner_features=(32, 8, 4))).train()
    assert list(model.state_dict().keys()) == list(g["gds::state_dict_keys"])
    x = torch.from_numpy(g["gds::x"])
    pred = model(x)
    close_map(pred, g["gds::train_pred"], 1e-4, "train-mode depth map")
    loss = ops.train_loss(pred, torch.from_numpy(g["gds::depth"]))
    close(loss, g["gds::train_loss"], rtol=1e-5)
    loss.backward()
    _check_grad_summary(model, g, "gds::", rtol=1e-2)
    model.eval()
    with torch.no_grad():
        close_map(model(x), g["gds::eval_pred"], 1e-4, "eval-mode depth map")


@pytest.mark.parametrize("tag", ["rand", "close", "anti"])
def test_ssim_matches_reference(golden, tag):
    g = golden("golden_losses.npz")
    x = torch.from_numpy(g[f"ssim_{tag}::x"]).requires_grad_(True)
    y = torch.from_numpy(g[f"ssim_{tag}::y"]).requires_grad_(True)
    v = ops.ssim3(x, y)
    close(v, g[f"ssim_{tag}::loss"], rtol=1e-5)
    v.backward()
    close(x.grad, g[f"ssim_{tag}::gx"], rtol=1e-4, atol=1e-8)
    close(y.grad, g[f"ssim_{tag}::gy"], rtol=1e-4, atol=1e-8)


def test_train_objective_matches_reference(golden):
    g = golden("golden_losses.npz")
    pred = torch.from_numpy(g["train::pred"]).requires_grad_(True)
    depth = torch.from_numpy(g["train::depth"])
    close(ops.depth_norm(depth), g["train::depth_n"], rtol=1e-6, atol=1e-7)
    dn = ops.depth_norm(depth)
    close(ops.l1(pred, dn), g["train::l1"])
    close(ops.ssim3(pred, dn), g["train::ssim"])
    close(ops.silog(pred, dn), g["train::silog"], rtol=1e-5)
    loss = ops.train_loss(pred, depth)
    close(loss, g["train::loss"])
    loss.backward()
    close(pred.grad, g["train::gpred"], rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("tag", ["dl_alh", "dl_mask", "dl_small", "dl_ssim_only"])
def test_depth_loss_matches_reference(golden, tag):
    g = golden("golden_losses.npz")
    a, b, gm, mx = (float(v) for v in g[f"{tag}::params"])
    x = torch.from_numpy(g[f"{tag}::pred"]).requires_grad_(True)
    v = ops.depth_loss(x, torch.from_numpy(g[f"{tag}::gt"]), a, b, gm, mx)
    close(v, g[f"{tag}::loss"], rtol=1e-5)
    v.backward()
    close(x.grad, g[f"{tag}::gpred"], rtol=1e-4, atol=1e-8)


def test_guidedepth_matches_reference(golden):
    g = golden("golden_guidedepth.npz")
    model = fill_(og.GuideDepth()).train()
    assert list(model.state_dict().keys()) == list(g["state_dict_keys"])
    x = torch.from_numpy(g["x"])
    pred = model(x)
    close_map(pred, g["train_pred"], 1e-4, "train-mode depth map")
    loss = ops.train_loss(pred, torch.from_numpy(g["depth"]))
    close(loss, g["train_loss"], rtol=1e-5)
    loss.backward()
    # Whole-network fp32 gradients of this randomly filled model are only good
    # to ~2e-3 (median relative error of BOTH the reference and the oracle vs
    # a float64 run of the oracle, measured): train-mode BN over 1x2 maps at
    # the bottom of DDRNet is ill-conditioned.  Hence 1e-2 here; the block and
    # op tests above pin the pieces at 1e-4.
    _check_grad_summary(model, g, "", rtol=1e-2)
    rm = [v for k, v in model.state_dict().items() if k.endswith("running_mean")]
    np.testing.assert_allclose([float(v.double().sum()) for v in rm], g["running_mean_sums"],
                               rtol=1e-4, atol=1e-6)
    model.eval()
    with torch.no_grad():
        close_map(model(x), g["eval_pred"], 1e-4, "eval-mode depth map")


def test_train_sequence_matches_reference(golden):
    """5 Adam steps of the train.py recipe incl. the eval-mode switch after step 0."""
    g = golden("golden_trainseq.npz")
    model = fill_(og.GuideDepth())
    opt = torch.optim.Adam(model.parameters(), 1e-4)
    model.train()
    losses = []
    for k in range(len(g["losses"])):
        image = torch.from_numpy(seeded((2, 3, 64, 96), 100 + k, 0, 1))
        depth = torch.from_numpy(seeded((2, 1, 64, 96), 200 + k, 0.1, 10.0))
        loss = ops.train_loss(model(image), depth)
        opt.zero_grad()
        losses.append(float(loss.detach()))
        loss.backward()
        opt.step()
        if k == 0:
            model.eval()
    # Step 0 is exact to 1e-6.  Adam's first update moves EVERY parameter by
    # ~lr * sign(g), including the conv biases in front of BatchNorm whose true
    # gradient is 0 (their sign is rounding noise); from step 1 on BN runs in
    # eval mode (train.py:161 quirk) where those biases matter, so the curves
    # agree only to the reference's own run-to-run sensitivity: up to 6.0e-3
    # from this golden when only the CPU thread count changes (1 thread).
    np.testing.assert_allclose(losses[0], g["losses"][0], rtol=1e-6)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-2)
    close_map(model.up_3.reduce.weight, g["final_up3_reduce_weight"], 1e-2, "up_3.reduce.weight")


def test_metrics_oracle_matches_reference(golden):
    """oracle/metrics.py vs the reference's compute_errors / Result.evaluate."""
    from oracle import metrics as om
    g = golden("golden_metrics.npz")
    np.testing.assert_allclose(om.batch_errors(g["metrics::gt"], g["metrics::pred"]),
                               g["metrics::batch"], rtol=1e-6)
    np.testing.assert_allclose(om.compute_errors(g["metrics::plain_gt"], g["metrics::plain_pred"]),
                               g["metrics::plain"], rtol=1e-6)
    r = om.fastdepth_evaluate(torch.from_numpy(g["metrics::fd_output"]),
                              torch.from_numpy(g["metrics::fd_target"]))
    np.testing.assert_allclose([r[f] for f in g["metrics::fd_fields"]], g["metrics::fd"], rtol=1e-6)
