"""Capture golden fixtures by importing the REFERENCE (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports LuizGuzzo/Monocular_Depth_Estimation from /root/reference/src
(read-only; no bytecode written), fills every module with the deterministic
weights of oracle/weights.py, runs the reference code on seeded inputs and
writes tests/golden/*.npz (inputs + expected outputs only — no reference
source travels).  cv2 is not installed here: an in-memory stub providing
INTER_CUBIC lets src/utils.py import (DepthNorm does not use cv2).  The
timm helpers newcrf_layers.py imports are stubbed the same way when NewCRF
fixtures are captured.

Exits if /root/reference is absent (e.g. on the GPU box): fixtures are
committed, the GPU box never re-captures.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"

sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from oracle.weights import fill_, seeded  # noqa: E402


def _import_reference():
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: golden fixtures can only be captured in the build container")
    if "cv2" not in sys.modules:
        cv2 = types.ModuleType("cv2")
        cv2.INTER_CUBIC = 2
        sys.modules["cv2"] = cv2
    # timm (absent) provides three helpers to newcrf_layers.py / SAM.py; every
    # drop_path rate on the path is 0, so DropPath is never instantiated, and
    # trunc_normal_ only initialises (fixtures overwrite all weights).
    if "timm" not in sys.modules:
        timm = types.ModuleType("timm")
        models = types.ModuleType("timm.models")
        layers = types.ModuleType("timm.models.layers")

        class DropPath(torch.nn.Module):
            def __init__(self, p=0.0):
                super().__init__()

            def forward(self, x):
                return x

        layers.DropPath = DropPath
        layers.to_2tuple = lambda v: tuple(v) if isinstance(v, (tuple, list)) else (v, v)
        layers.trunc_normal_ = lambda t, std=1.0: torch.nn.init.trunc_normal_(t, std=std, a=-2.0, b=2.0)
        timm.models, models.layers = models, layers
        sys.modules.update({"timm": timm, "timm.models": models, "timm.models.layers": layers})
    # torchvision (absent) is only touched by Encoder(), which is not captured
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tv.models = types.ModuleType("torchvision.models")
        sys.modules.update({"torchvision": tv, "torchvision.models": tv.models})
    sys.path.insert(0, REF)
    os.chdir(REF)  # GuideDepth package imports are relative to src/


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def grad_summary(module, prefix, out, full_limit=4096, force=()):
    """Per-parameter grad sum and L2 norm; full grads for small / forced params."""
    names, sums, norms = [], [], []
    for name, p in module.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().double()
        names.append(name)
        sums.append(float(g.sum()))
        norms.append(float(g.norm()))
        if p.numel() <= full_limit or name in force:
            out[f"{prefix}grad::{name}"] = f32(p.grad)
    out[f"{prefix}grad_names"] = np.array(names)
    out[f"{prefix}grad_sums"] = np.array(sums, dtype=np.float64)
    out[f"{prefix}grad_norms"] = np.array(norms, dtype=np.float64)


RESIZE_CASES = [
    # name, shape, kwargs
    ("b_30x40_to_60x80", (1, 2, 30, 40), dict(size=[60, 80])),
    ("b_15x20_to_60x80", (1, 2, 15, 20), dict(size=[60, 80])),
    ("b_4x5_to_8x10", (1, 2, 4, 5), dict(size=[8, 10])),
    ("b_2x3_to_8x10", (1, 2, 2, 3), dict(size=[8, 10])),
    ("b_1x2_to_8x10", (1, 2, 1, 2), dict(size=[8, 10])),
    ("b_1x1_to_8x10", (1, 2, 1, 1), dict(size=[8, 10])),
    ("b_8x10_to_60x80", (1, 2, 8, 10), dict(size=[60, 80])),
    ("b_8x10_to_30x40", (1, 2, 8, 10), dict(size=[30, 40])),
    ("b_x2", (2, 3, 16, 20), dict(scale_factor=2)),
    ("b_x2_odd", (1, 2, 7, 9), dict(scale_factor=2)),
    ("b_align_x2", (1, 2, 7, 9), dict(scale_factor=2, align_corners=True)),
    ("b_align_size", (1, 2, 5, 6), dict(size=[11, 17], align_corners=True)),
    ("b_down_20x30_to_7x11", (1, 2, 20, 30), dict(size=[7, 11])),
    ("b_5x7_to_13x17", (1, 1, 5, 7), dict(size=[13, 17])),
    ("b_x4", (1, 1, 6, 8), dict(scale_factor=4)),
]
NEAREST_CASES = [
    ("n_half", (1, 3, 24, 32), 0.5),
    ("n_quarter", (1, 3, 24, 32), 0.25),
    ("n_half_odd", (1, 3, 25, 33), 0.5),
    ("n_quarter_odd", (1, 3, 27, 35), 0.25),
]


def capture_resize():
    import torch.nn.functional as F
    out = {}
    for i, (name, shape, kw) in enumerate(RESIZE_CASES):
        x = torch.from_numpy(seeded(shape, 1000 + i, -1, 1)).requires_grad_(True)
        y = F.interpolate(x, mode="bilinear", **kw)
        gy = torch.from_numpy(seeded(y.shape, 2000 + i, -1, 1))
        y.backward(gy)
        out.update({f"{name}::x": f32(x), f"{name}::gy": f32(gy), f"{name}::y": f32(y),
                    f"{name}::gx": f32(x.grad)})
    for i, (name, shape, sf) in enumerate(NEAREST_CASES):
        x = torch.from_numpy(seeded(shape, 3000 + i, -1, 1)).requires_grad_(True)
        y = F.interpolate(x, scale_factor=sf)
        gy = torch.from_numpy(seeded(y.shape, 4000 + i, -1, 1))
        y.backward(gy)
        out.update({f"{name}::x": f32(x), f"{name}::gy": f32(gy), f"{name}::y": f32(y),
                    f"{name}::gx": f32(x.grad)})
    return out


def capture_blocks():
    from GuideDepth.model.modules import Guided_Upsampling_Block, SELayer
    out = {}
    # SELayer(16, reduction=1) as used inside up_3, plus a reduction-4 case
    for tag, ch, red, shape in (("se16", 16, 1, (2, 16, 10, 12)), ("se32r4", 32, 4, (2, 32, 6, 7))):
        m = fill_(SELayer(ch, reduction=red))
        x = torch.from_numpy(seeded(shape, 11, -1, 1)).requires_grad_(True)
        y = m(x)
        gy = torch.from_numpy(seeded(y.shape, 12, -1, 1))
        y.backward(gy)
        out.update({f"{tag}::x": f32(x), f"{tag}::gy": f32(gy), f"{tag}::y": f32(y),
                    f"{tag}::gx": f32(x.grad), f"{tag}::gw1": f32(m.fc[0].weight.grad),
                    f"{tag}::gw2": f32(m.fc[2].weight.grad)})
    # the three guided-upsampling configurations of GuideDepth, train-mode BN
    for tag, (cin, e, cout) in (("gub1", (64, 64, 32)), ("gub2", (32, 32, 16)),
                                ("gub3", (16, 16, 1))):
        m = fill_(Guided_Upsampling_Block(cin, e, cout, kernel_size=3, channel_attention=True,
                                          guide_features=3, guidance_type="full"))
        m.train()
        guide = torch.from_numpy(seeded((2, 3, 12, 16), 21, 0, 1)).requires_grad_(True)
        depth = torch.from_numpy(seeded((2, cin, 12, 16), 22, -1, 1)).requires_grad_(True)
        y = m(guide, depth)
        gy = torch.from_numpy(seeded(y.shape, 23, -1, 1))
        y.backward(gy)
        out.update({f"{tag}::guide": f32(guide), f"{tag}::depth": f32(depth),
                    f"{tag}::gy": f32(gy), f"{tag}::y": f32(y),
                    f"{tag}::gguide": f32(guide.grad), f"{tag}::gdepth": f32(depth.grad)})
        grad_summary(m, f"{tag}::", out, full_limit=2048)
    return out


# reference API variants (modules.py:62-65,80,91-96; loader.py:18-19):
# tag -> (in, expand, out, channel_attention, guidance_type)
VARIANT_BLOCKS = {
    "gub_raw": (16, 16, 1, True, "raw"),
    "gub_none": (16, 16, 1, True, "none"),
    "gub_noca": (32, 32, 16, False, "full"),
    "gub_raw_noca": (32, 32, 16, False, "raw"),
    "gub_none_noca": (64, 64, 32, False, "none"),
}


def capture_variants():
    """Guided_Upsampling_Block's non-default guidance types / no channel
    attention, and GuideDepth-S (up / inner features [32, 8, 4])."""
    from GuideDepth.model.GuideDepth import GuideDepth
    from GuideDepth.model.modules import Guided_Upsampling_Block
    import loss as refloss
    import utils as refutils
    out = {}
    for i, (tag, (cin, e, cout, ca, gt)) in enumerate(VARIANT_BLOCKS.items()):
        m = fill_(Guided_Upsampling_Block(cin, e, cout, kernel_size=3, channel_attention=ca,
                                          guide_features=3, guidance_type=gt))
        m.train()
        guide = torch.from_numpy(seeded((2, 3, 12, 16), 121 + i, 0, 1)).requires_grad_(True)
        depth = torch.from_numpy(seeded((2, cin, 12, 16), 131 + i, -1, 1)).requires_grad_(True)
        y = m(guide, depth)
        gy = torch.from_numpy(seeded(y.shape, 141 + i, -1, 1))
        y.backward(gy)
        out.update({f"{tag}::guide": f32(guide), f"{tag}::depth": f32(depth),
                    f"{tag}::gy": f32(gy), f"{tag}::y": f32(y), f"{tag}::gdepth": f32(depth.grad),
                    f"{tag}::cfg": np.array([cin, e, cout, int(ca)], dtype=np.int64),
                    f"{tag}::guidance": np.array(gt)})
        if guide.grad is not None:  # 'none' never reads the guide
            out[f"{tag}::gguide"] = f32(guide.grad)
        grad_summary(m, f"{tag}::", out, full_limit=2048)
    # GuideDepth-S (loader.py:18-19), train-mode step objective + eval map
    model = fill_(GuideDepth(pretrained=False, up_features=[32, 8, 4], inner_features=[32, 8, 4]))
    out["gds::state_dict_keys"] = np.array(list(model.state_dict().keys()))
    x = torch.from_numpy(seeded((2, 3, 128, 192), 161, 0, 1))  # 64x96 leaves DDRNet BN over 2 values: ill-conditioned
    depth = torch.from_numpy(seeded((2, 1, 128, 192), 162, 0.1, 10.0))
    model.train()
    pred = model(x)
    dn = refutils.DepthNorm(depth)
    loss = 1.0 * refloss.SSIM()(pred, dn) + 0.1 * torch.nn.L1Loss()(pred, dn)
    loss.backward()
    out.update({"gds::x": f32(x), "gds::depth": f32(depth), "gds::train_pred": f32(pred),
                "gds::train_loss": f32(loss)})
    grad_summary(model, "gds::", out, full_limit=512)
    model.eval()
    with torch.no_grad():
        out["gds::eval_pred"] = f32(model(x))
    return out


def capture_losses():
    import loss as refloss
    import utils as refutils
    from GuideDepth.losses import Depth_Loss
    out = {}
    shape = (2, 1, 24, 32)
    cases = {
        "rand": (seeded(shape, 31, 0, 1), seeded(shape, 32, 0, 1)),
        "close": (None, seeded(shape, 33, 0, 1)),
        "anti": (None, seeded(shape, 34, 0, 1)),
    }
    cases["close"] = (cases["close"][1] + 0.01 * seeded(shape, 35, -1, 1), cases["close"][1])
    cases["anti"] = (1.0 - cases["anti"][1], cases["anti"][1])
    ssim = refloss.SSIM()
    for tag, (p, t) in cases.items():
        x = torch.from_numpy(p).requires_grad_(True)
        y = torch.from_numpy(t).requires_grad_(True)
        v = ssim(x, y)
        v.backward()
        out.update({f"ssim_{tag}::x": p, f"ssim_{tag}::y": t, f"ssim_{tag}::loss": f32(v),
                    f"ssim_{tag}::gx": f32(x.grad), f"ssim_{tag}::gy": f32(y.grad)})
    # train.py objective: DepthNorm target, SSIM + 0.1 L1 (train.py:89-100)
    pred = torch.from_numpy(seeded(shape, 41, 0, 1)).requires_grad_(True)
    depth = torch.from_numpy(seeded(shape, 42, 0.1, 10.0))
    dn = refutils.DepthNorm(depth)
    l1 = torch.nn.L1Loss()(pred, dn)
    ls = ssim(pred, dn)
    sil = refloss.Silog_loss_variance()(pred, dn)
    total = 1.0 * ls + 0.1 * l1
    total.backward()
    out.update({"train::pred": f32(pred), "train::depth": f32(depth), "train::depth_n": f32(dn),
                "train::l1": f32(l1), "train::ssim": f32(ls), "train::silog": f32(sil),
                "train::loss": f32(total), "train::gpred": f32(pred.grad)})
    # Depth_Loss in Alhashim mode (0.1,1,1), masked L1 mode (1,0,0) and a small map (K=8)
    for tag, (a, b, g), shp, mx in (("dl_alh", (0.1, 1.0, 1.0), (2, 1, 24, 32), 10.0),
                                    ("dl_mask", (1.0, 0.0, 0.0), (2, 1, 24, 32), 10.0),
                                    ("dl_small", (0.1, 1.0, 1.0), (1, 1, 8, 9), 10.0),
                                    ("dl_ssim_only", (0.0, 1.0, 0.0), (1, 2, 16, 20), 1.0)):
        p = seeded(shp, 51, 0.0, mx)
        t = seeded(shp, 52, 0.0, mx)
        if tag == "dl_mask":
            t[..., ::3, ::2] = 0.0  # invalid pixels
        x = torch.from_numpy(p).requires_grad_(True)
        v = Depth_Loss(a, b, g, maxDepth=mx)(x, torch.from_numpy(t))
        v.backward()
        out.update({f"{tag}::pred": p, f"{tag}::gt": t, f"{tag}::loss": f32(v),
                    f"{tag}::gpred": f32(x.grad),
                    f"{tag}::params": np.array([a, b, g, mx], dtype=np.float32)})
    return out


def capture_guidedepth():
    from GuideDepth.model.GuideDepth import GuideDepth
    import loss as refloss
    import utils as refutils
    out = {}
    model = fill_(GuideDepth(pretrained=False))
    out["state_dict_keys"] = np.array(list(model.state_dict().keys()))
    x = torch.from_numpy(seeded((2, 3, 64, 96), 61, 0, 1))
    depth = torch.from_numpy(seeded((2, 1, 64, 96), 62, 0.1, 10.0))
    feats = {}
    hooks = [getattr(model, n).register_forward_hook(
        lambda m, i, o, n=n: feats.__setitem__(n, o.detach().clone())) for n in ("up_1", "up_2")]
    hooks.append(model.feature_extractor.register_forward_hook(
        lambda m, i, o: feats.__setitem__("encoder", o.detach().clone())))
    model.train()
    pred = model(x)
    for h in hooks:
        h.remove()
    dn = refutils.DepthNorm(depth)
    loss = 1.0 * refloss.SSIM()(pred, dn) + 0.1 * torch.nn.L1Loss()(pred, dn)
    loss.backward()
    out.update({"x": f32(x), "depth": f32(depth), "train_pred": f32(pred), "train_loss": f32(loss)})
    for k, v in feats.items():
        out[f"train_{k}"] = f32(v)
    grad_summary(model, "", out, full_limit=2048, force=("feature_extractor.conv1.0.weight",))
    rm = [v for k, v in model.state_dict().items() if k.endswith("running_mean")]
    out["running_mean_sums"] = np.array([float(v.double().sum()) for v in rm])
    model.eval()
    with torch.no_grad():
        out["eval_pred"] = f32(model(x))
    return out


def capture_train_sequence(steps=5):
    """train.py recipe (train.py:79-136): step 0 in train mode, then LogProgress's
    model.eval() sticks (train.py:161) for the rest of the epoch."""
    from GuideDepth.model.GuideDepth import GuideDepth
    import loss as refloss
    import utils as refutils
    model = fill_(GuideDepth(pretrained=False))
    opt = torch.optim.Adam(model.parameters(), 1e-4)
    l1, ssim = torch.nn.L1Loss(), refloss.SSIM()
    model.train()
    losses = []
    for k in range(steps):
        image = torch.from_numpy(seeded((2, 3, 64, 96), 100 + k, 0, 1))
        depth = torch.from_numpy(seeded((2, 1, 64, 96), 200 + k, 0.1, 10.0))
        dn = refutils.DepthNorm(depth)
        pred = model(image)
        loss = 1.0 * ssim(pred, dn) + 0.1 * l1(pred, dn)
        opt.zero_grad()
        losses.append(float(loss.item()))
        loss.backward()
        opt.step()
        if k == 0:
            model.eval()  # LogProgress at loader_pos % 300 == 0
    return {"losses": np.array(losses, dtype=np.float64),
            "final_up3_reduce_weight": f32(model.up_3.reduce.weight)}


NEWCRF_CASES = [
    # tag, (input_dim, embed_dim, v_dim, heads), batch, (h, w)
    ("crf0", (24, 128, 64, 4), 2, (10, 13)),
    ("crf1", (40, 256, 128, 8), 2, (7, 9)),
    ("crf2", (112, 512, 256, 16), 1, (8, 9)),
    ("crf3", (160, 1024, 512, 32), 1, (5, 6)),
    ("crf_same_v", (64, 64, 64, 2), 2, (14, 7)),  # multiples of 7, no proj_v
]


def capture_newcrf():
    from newcrf_layers import NewCRF
    out = {}
    for tag, (ind, emb, vd, heads), b, (h, w) in NEWCRF_CASES:
        m = fill_(NewCRF(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads))
        x = torch.from_numpy(seeded((b, ind, h, w), 81, -1, 1)).requires_grad_(True)
        v = torch.from_numpy(seeded((b, vd, h, w), 82, -1, 1)).requires_grad_(True)
        y = m(x, v)
        gy = torch.from_numpy(seeded(y.shape, 83, -1, 1))
        y.backward(gy)
        out.update({f"{tag}::x": f32(x), f"{tag}::v": f32(v), f"{tag}::gy": f32(gy),
                    f"{tag}::y": f32(y), f"{tag}::gx": f32(x.grad), f"{tag}::gv": f32(v.grad)})
        out[f"{tag}::keys"] = np.array(list(m.state_dict().keys()))
        grad_summary(m, f"{tag}::", out, full_limit=1024)
    # the full Decoder on the feature pyramid of a 64x96 image (feats 4, 7, 13, 16, 17)
    from model_mobileV3_large_newCRFs import Decoder
    dec = fill_(Decoder())
    shapes = {4: (24, 16, 24), 7: (40, 8, 12), 13: (112, 4, 6), 16: (160, 2, 3), 17: (960, 2, 3)}
    feats = [None] * 18
    for i, (c, h, w) in shapes.items():
        feats[i] = torch.from_numpy(seeded((2, c, h, w), 90 + i, -1, 1)).requires_grad_(True)
    y = dec(feats)
    gy = torch.from_numpy(seeded(y.shape, 99, -1, 1))
    y.backward(gy)
    out["dec::keys"] = np.array(list(dec.state_dict().keys()))
    out["dec::y"], out["dec::gy"] = f32(y), f32(gy)
    for i in shapes:
        out[f"dec::feat{i}"] = f32(feats[i])
        out[f"dec::gfeat{i}"] = f32(feats[i].grad)
    grad_summary(dec, "dec::", out, full_limit=1024)
    return out


SAM_CASES = [
    # tag, (input_dim, embed_dim, v_dim, heads), batch, (h, w)   (SAM.forward(e, q): e has
    # input_dim channels, q has v_dim)
    ("sam0", (24, 128, 64, 4), 2, (10, 13)),
    ("sam1", (40, 256, 128, 8), 1, (8, 12)),
    ("sam3", (160, 1024, 512, 32), 1, (3, 5)),
    ("sam_same", (64, 64, 64, 2), 2, (14, 7)),  # multiples of 7, no projections
]


def capture_sam():
    """src/SAM.py SAM stages and the model_mobileV3_large_SAM.py Decoder, fwd + bwd."""
    from SAM import SAM
    out = {}
    for tag, (ind, emb, vd, heads), b, (h, w) in SAM_CASES:
        m = fill_(SAM(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads))
        e = torch.from_numpy(seeded((b, ind, h, w), 71, -1, 1)).requires_grad_(True)
        q = torch.from_numpy(seeded((b, vd, h, w), 72, -1, 1)).requires_grad_(True)
        y = m(e, q)
        gy = torch.from_numpy(seeded(y.shape, 73, -1, 1))
        y.backward(gy)
        out.update({f"{tag}::e": f32(e), f"{tag}::q": f32(q), f"{tag}::gy": f32(gy),
                    f"{tag}::y": f32(y), f"{tag}::ge": f32(e.grad), f"{tag}::gq": f32(q.grad)})
        out[f"{tag}::keys"] = np.array(list(m.state_dict().keys()))
        grad_summary(m, f"{tag}::", out, full_limit=1024)
    from model_mobileV3_large_SAM import Decoder
    dec = fill_(Decoder())
    shapes = {4: (24, 16, 24), 7: (40, 8, 12), 13: (112, 4, 6), 16: (160, 2, 3), 17: (960, 2, 3)}
    feats = [None] * 18
    for i, (c, h, w) in shapes.items():
        feats[i] = torch.from_numpy(seeded((2, c, h, w), 60 + i, -1, 1)).requires_grad_(True)
    y = dec(feats)
    gy = torch.from_numpy(seeded(y.shape, 69, -1, 1))
    y.backward(gy)
    out["dec::keys"] = np.array(list(dec.state_dict().keys()))
    out["dec::y"], out["dec::gy"] = f32(y), f32(gy)
    for i in shapes:
        out[f"dec::feat{i}"] = f32(feats[i])
        out[f"dec::gfeat{i}"] = f32(feats[i].grad)
    grad_summary(dec, "dec::", out, full_limit=1024)
    return out


def capture_metrics():
    """utils.compute_errors (src/utils.py:45-66) on the pixels src/test.py:105-118
    keeps (clamp / range mask / Eigen crop, restated inline as test.py is a
    script), on plain positive arrays, and GuideDepth/metrics.py Result.evaluate."""
    import utils as refutils
    from GuideDepth.metrics import Result
    out = {}
    rng = np.random.default_rng(7)
    n, h, w = 3, 48, 64
    depth = torch.from_numpy(rng.uniform(0.1, 10.0, (n, 1, h, w)).astype(np.float32))
    gt = refutils.DepthNorm(depth).numpy().squeeze()          # test.py:91,100
    gt[0, 10:14, 10:20] = 0.0005                               # below min_depth_eval
    pred = rng.uniform(-0.05, 1.1, (n, h, w)).astype(np.float32)
    pred[1, 20, 5:9] = [np.inf, -np.inf, np.nan, 100.0]
    pred[2, 30, 30] = np.nan
    out["metrics::gt"], out["metrics::pred"] = gt.copy(), pred.copy()
    lo, hi = 1e-3, 80.0                                        # test.py:34-35 defaults
    p = pred.copy()
    p[p < lo] = lo
    p[p > hi] = hi
    p[np.isinf(p)] = hi
    p[np.isnan(p)] = lo
    mask = np.logical_and(gt > lo, gt < hi)
    crop = np.array([int(0.09375 * h), int(0.98125 * h), int(0.0640625 * w),
                     int(0.9390625 * w)]).astype(np.int32)
    cm = np.zeros(mask.shape)
    cm[:, crop[0]:crop[1], crop[2]:crop[3]] = 1
    mask = np.logical_and(mask, cm)
    out["metrics::batch"] = np.array(refutils.compute_errors(gt[mask], p[mask]), dtype=np.float64)
    g2 = rng.uniform(0.05, 10.0, 5000).astype(np.float32)
    p2 = (g2 * rng.uniform(0.6, 1.6, 5000)).astype(np.float32)
    out["metrics::plain_gt"], out["metrics::plain_pred"] = g2, p2
    out["metrics::plain"] = np.array(refutils.compute_errors(g2, p2), dtype=np.float64)
    t = torch.from_numpy(rng.uniform(0.1, 10.0, (2, 1, 24, 32)).astype(np.float32))
    o = (t * torch.from_numpy(rng.uniform(0.7, 1.4, (2, 1, 24, 32)).astype(np.float32)))
    r = Result()
    r.evaluate(o, t)
    out["metrics::fd_output"], out["metrics::fd_target"] = f32(o), f32(t)
    fields = ("mse", "rmse", "mae", "lg10", "rmse_log", "absrel", "delta1", "delta2", "delta3",
              "irmse", "imae")
    out["metrics::fd_fields"] = np.array(fields)
    out["metrics::fd"] = np.array([float(getattr(r, f)) for f in fields], dtype=np.float64)
    return out


def _nyu_zip(path, n_train=12, n_test=5, h=6, w=10):
    """A miniature CSVdata.zip: data/nyu2_{train,test}.csv + RGB JPEG-free PNG pairs."""
    import zipfile
    from PIL import Image
    rng = np.random.default_rng(5)
    rows = {"train": [], "test": []}
    with zipfile.ZipFile(path, "w") as z:
        for split, count in (("train", n_train), ("test", n_test)):
            for i in range(count):
                a = f"data/nyu2_{split}/scene_{i % 3}/{i}.png"
                b = f"data/nyu2_{split}/scene_{i % 3}/{i}_depth.png"
                for name, arr in ((a, rng.integers(0, 256, (h, w, 3), dtype=np.uint8)),
                                  (b, rng.integers(0, 256, (h, w), dtype=np.uint8))):
                    buf = __import__("io").BytesIO()
                    Image.fromarray(arr).save(buf, format="PNG")
                    z.writestr(name, buf.getvalue())
                rows[split].append(f"{a},{b}")
            z.writestr(f"data/nyu2_{split}.csv", "\n".join(rows[split]) + "\n")
    return rows


def capture_data():
    """src/data.py: getDefaultTrainTransform / getNoTransform on seeded `random`
    draws (torchvision.transforms.Compose stubbed: data.py only composes), and
    loadZipToMem's shuffled train / test rows on a miniature zip."""
    import random as pyrandom
    import tempfile
    from PIL import Image
    tv = sys.modules.get("torchvision") or types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, s):
            for t in self.ts:
                s = t(s)
            return s

    tr.Compose = Compose
    tv.transforms, tv.utils = tr, types.ModuleType("torchvision.utils")
    sys.modules["torchvision"], sys.modules["torchvision.transforms"] = tv, tr
    sys.modules["torchvision.utils"] = tv.utils
    import data as refdata
    out = {}
    rng = np.random.default_rng(9)
    imgs = rng.integers(0, 256, (2, 6, 10, 3), dtype=np.uint8)
    deps = rng.integers(0, 256, (2, 6, 10), dtype=np.uint8)
    out["data::img"], out["data::dep"] = imgs, deps
    seeds = np.arange(100, 116)
    out["data::seeds"] = seeds
    for i, sd in enumerate(seeds):
        pyrandom.seed(int(sd))
        s = refdata.getDefaultTrainTransform()({"image": Image.fromarray(imgs[i % 2]),
                                                "depth": Image.fromarray(deps[i % 2])})
        out[f"data::train{i}::image"], out[f"data::train{i}::depth"] = f32(s["image"]), f32(s["depth"])
    s = refdata.getNoTransform()({"image": Image.fromarray(imgs[0]), "depth": Image.fromarray(deps[0])})
    out["data::test::image"], out["data::test::depth"] = f32(s["image"]), f32(s["depth"])
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "CSVdata.zip")
        _nyu_zip(path)
        _, train, test = refdata.loadZipToMem(path)
    out["data::zip_train"] = np.array([",".join(r) for r in train])
    out["data::zip_test"] = np.array([",".join(r) for r in test])
    return out


def main():
    _import_reference()
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    jobs = {"golden_resize.npz": capture_resize, "golden_blocks.npz": capture_blocks,
            "golden_losses.npz": capture_losses, "golden_guidedepth.npz": capture_guidedepth,
            "golden_trainseq.npz": capture_train_sequence, "golden_newcrf.npz": capture_newcrf,
            "golden_metrics.npz": capture_metrics, "golden_data.npz": capture_data,
            "golden_sam.npz": capture_sam, "golden_variants.npz": capture_variants}
    only = set(sys.argv[1:])
    for fname, fn in jobs.items():
        if only and fname not in only:
            continue
        data = fn()
        path = os.path.join(HERE, fname)
        np.savez_compressed(path, **data)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB, {len(data)} arrays)")


if __name__ == "__main__":
    main()
