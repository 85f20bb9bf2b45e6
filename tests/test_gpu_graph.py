"""HIP-graph training step (GraphTrainer) == eager step (Trainer), GuideDepth and PTModel.

Same init, same batches, BN in train mode, 6 steps (2 eager warm-up,
capture, 3 replays).  MIOpen's default convolution solvers are not bitwise
run-to-run deterministic (two EAGER runs of GuideDepth differ by ~1e-7 in the
loss and, through Adam's sign-like first update, by lr-sized steps on
near-zero gradients), so the test selects its deterministic solvers
(torch.backends.cudnn.deterministic): then two eager runs are bitwise equal
and the graph run must match the eager run to 1e-6 in every loss and every
parameter.  Every step must also have moved the parameters (the graph really
trains).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    yield
    torch.backends.cudnn.deterministic = old


def _run(build, graph, steps=6, bs=2, h=64, w=96, amp=""):
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import (GraphTrainer, Trainer, World, make_adam,
                                                      synthetic_batch)
    torch.manual_seed(0)
    model = build().to(DEV)
    world = World(0, 0, 1, torch.device(DEV))
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    if graph:
        tr = GraphTrainer(model, loss_fn, world, lr=1e-4, amp=amp)
    else:
        tr = Trainer(model, make_adam(model, 1e-4), loss_fn, world, eval_quirk=False, amp=amp)
    tr.begin_epoch()
    losses, moved = [], []
    for k in range(steps):
        before = torch.cat([p.detach().flatten() for p in model.parameters()]).clone()
        image, depth = synthetic_batch(bs, h, w, 0, k, DEV)
        losses.append(float(tr.step(image, depth).detach()))
        after = torch.cat([p.detach().flatten() for p in model.parameters()])
        moved.append(float((after - before).abs().max()))
    torch.cuda.synchronize()
    return losses, moved, {n: p.detach().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("which", ["guidedepth", "ptmodel"])
def test_graph_step_matches_eager(which):
    if which == "guidedepth":
        from monocular_depth_estimation_amd import GuideDepth
        build = lambda: GuideDepth(pretrained=False)  # noqa: E731
    else:
        from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
        build = PTModel
    le, _, pe = _run(build, graph=False)
    lg, moved, pg = _run(build, graph=True)
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-6 * abs(b), (lg, le)
    worst = max(float((pg[n] - pe[n]).abs().max()) for n in pe)
    assert worst <= 1e-6, worst
    assert min(moved) > 0.5e-4, moved  # Adam moves weights by ~lr = 1e-4 every step


def test_bf16_autocast_step():
    """BASELINE cfg3 precision: convs / GEMMs autocast to bf16, the HIP kernels
    take fp32 (their Functions cast); the graph replays the autocast step like
    the eager one, and the losses track the fp32 run to bf16 accuracy."""
    from monocular_depth_estimation_amd import GuideDepth
    build = lambda: GuideDepth(pretrained=False)  # noqa: E731
    lf, _, _ = _run(build, graph=False)
    le, _, pe = _run(build, graph=False, amp="bf16")
    lg, moved, pg = _run(build, graph=True, amp="bf16")
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-5 * abs(b), (lg, le)
    worst = max(float((pg[n] - pe[n]).abs().max()) for n in pe)
    assert worst <= 1e-5, worst
    for a, b in zip(le, lf):  # bf16 products (8-bit mantissa) vs fp32
        assert abs(a - b) <= 3e-2 * abs(b), (le, lf)
    assert min(moved) > 0.5e-4, moved
