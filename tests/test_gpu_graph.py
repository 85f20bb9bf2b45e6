"""HIP-graph training step (GraphTrainer) == eager step (Trainer), GuideDepth and PTModel.

Same init, same batches, BN in train mode: the losses of 6 steps (2 eager
warm-up, capture, 3 replays) and the final parameters must match the eager
Trainer to 1e-5 (fused capturable Adam vs fused Adam: same update rule, the
step counter lives on the device).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


def _run(build, graph, steps=6, bs=2, h=64, w=96):
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import (GraphTrainer, Trainer, World, make_adam,
                                                      synthetic_batch)
    torch.manual_seed(0)
    model = build().to(DEV)
    world = World(0, 0, 1, torch.device(DEV))
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    if graph:
        tr = GraphTrainer(model, loss_fn, world, lr=1e-4)
    else:
        tr = Trainer(model, make_adam(model, 1e-4), loss_fn, world, eval_quirk=False)
    tr.begin_epoch()
    losses = []
    for k in range(steps):
        image, depth = synthetic_batch(bs, h, w, 0, k, DEV)
        losses.append(float(tr.step(image, depth)))
    torch.cuda.synchronize()
    return losses, {n: p.detach().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("which", ["guidedepth", "ptmodel"])
def test_graph_step_matches_eager(which):
    if which == "guidedepth":
        from monocular_depth_estimation_amd import GuideDepth
        build = lambda: GuideDepth(pretrained=False)  # noqa: E731
    else:
        from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
        build = PTModel
    le, pe = _run(build, graph=False)
    lg, pg = _run(build, graph=True)
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-5 * abs(b), (lg, le)
    worst = max(float((pg[n] - pe[n]).abs().max()) for n in pe)
    assert worst <= 1e-5, worst
