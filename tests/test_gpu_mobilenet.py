"""GPU parity of MobileNetV3-Large and the full NewCRF PTModel (cfg4 path) vs the CPU oracle.

The encoder's oracle (oracle/mobilenetv3.py) is a restatement of torchvision's
published architecture — parity UNPINNED against torchvision itself (absent
here); the decoder half is pinned by the reference goldens
(test_gpu_newcrf.py::test_decoder_golden).  Truth is the oracle run in
float64; the HIP fp32 path must sit within 1e-3 scale-relative on the depth
map (BASELINE north_star) and 1e-2 on parameter-gradient norms (fp32
conditioning of train-mode BatchNorm on small maps, as for GuideDepth).
"""
import numpy as np
import pytest
import torch

from oracle import mobilenetv3 as om
from oracle.weights import fill_, seeded

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


def close_scaled(a, b, tol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = float((a - b).abs().max())
    assert err <= tol * float(b.abs().max()) + 1e-30, f"{what}: {err:.3g} vs {float(b.abs().max()):.3g}"


def _pair(ours_cls, oracle_cls):
    ref = fill_(oracle_cls()).double().train()
    ours = ours_cls()
    ours.load_state_dict({k: v.float() if v.is_floating_point() else v
                          for k, v in ref.state_dict().items()})
    return ours.to(DEV).train(), ref


def _grad_norm_check(ours, ref, tol_max, tol_med):
    got, want = dict(ours.named_parameters()), dict(ref.named_parameters())
    errs = []
    for k, p in want.items():
        if p.grad is None:
            assert got[k].grad is None or float(got[k].grad.abs().max()) == 0.0, k
            continue
        w = float(p.grad.norm())
        if w < 1e-7 * max(float(q.grad.norm()) for q in want.values() if q.grad is not None):
            continue
        errs.append(abs(float(got[k].grad.double().norm()) - w) / w)
    errs = np.array(errs)
    assert errs.max() <= tol_max and np.median(errs) <= tol_med, (errs.max(), np.median(errs))


def test_encoder_features_vs_oracle():
    from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import Encoder
    ours, ref = _pair(Encoder, om.Encoder)
    x = torch.from_numpy(seeded((2, 3, 128, 160), 11, 0, 1))
    fo = ours(x.to(DEV))
    fr = ref(x.double())
    assert len(fo) == len(fr) == 18
    for i, (a, b) in enumerate(zip(fo, fr)):
        assert a.shape == b.shape, (i, a.shape, b.shape)
        close_scaled(a, b, 1e-3, f"feat{i}")
    # backward through the five features the decoder consumes
    loss_o = sum((fo[i] * (0.1 * (i + 1))).sum() for i in (4, 7, 13, 16, 17))
    loss_r = sum((fr[i] * (0.1 * (i + 1))).sum() for i in (4, 7, 13, 16, 17))
    loss_o.backward()
    loss_r.backward()
    _grad_norm_check(ours, ref, 1.5e-2, 5e-3)
    for k, v in ref.state_dict().items():
        if "running" in k:
            close_scaled(ours.state_dict()[k], v, 1e-4, k)


def test_ptmodel_step_vs_oracle():
    """One cfg4-shaped training step (forward, SSIM+0.1 L1 on DepthNorm'd target, backward)."""
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
    from oracle import ops as oops
    ours, ref = _pair(PTModel, om.PTModel)
    x = torch.from_numpy(seeded((2, 3, 128, 160), 21, 0, 1))
    d = torch.from_numpy(seeded((2, 1, 128, 160), 22, 0.5, 10))
    pred = ours(x.to(DEV))
    pr = ref(x.double())
    assert pred.shape == (2, 1, 128, 160)
    close_scaled(pred, pr, 1e-3, "depth map")
    loss = SSIML1()(pred, d.to(DEV))
    lr = oops.train_loss(pr, d.double())
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-4 * abs(float(lr))
    loss.backward()
    lr.backward()
    _grad_norm_check(ours, ref, 1.5e-2, 5e-3)


@pytest.mark.parametrize("n,c,cr,h,w", [(16, 72, 24, 60, 80), (2, 960, 240, 15, 20), (3, 120, 32, 7, 5)])
def test_se_hardsigmoid_vs_torch(n, c, cr, h, w):
    """torchvision SqueezeExcitation restated in float64 torch ops vs the HIP gated SE."""
    from monocular_depth_estimation_amd.mobilenetv3 import SqueezeExcitation
    se = SqueezeExcitation(c, cr)
    with torch.no_grad():
        se.fc1.weight.copy_(torch.from_numpy(seeded((cr, c, 1, 1), 1, -0.3, 0.3)))
        se.fc1.bias.copy_(torch.from_numpy(seeded((cr,), 2, -0.3, 0.3)))
        se.fc2.weight.copy_(torch.from_numpy(seeded((c, cr, 1, 1), 3, -0.6, 0.6)))
        se.fc2.bias.copy_(torch.from_numpy(seeded((c,), 4, -2, 2)))
    ref = om.SE(c, cr).double()
    ref.load_state_dict({k: v.double() for k, v in se.state_dict().items()})
    x = torch.from_numpy(seeded((n, c, h, w), 5, -1, 3))
    gy = torch.from_numpy(seeded((n, c, h, w), 6, -1, 1))
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy.double())
    se = se.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = se(xd)
    close_scaled(y, yr, 1e-5, "y")
    y.backward(gy.to(DEV))
    close_scaled(xd.grad, xr.grad, 1e-5, "gx")
    for name in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"):
        got = dict(se.named_parameters())[name].grad
        want = dict(ref.named_parameters())[name].grad
        close_scaled(got, want, 1e-4, name)
