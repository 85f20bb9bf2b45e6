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


def test_captured_memset_repaired():
    """A hipMemsetAsync captured into a graph is wrong from the second replay on
    (ROCm runtime; csrc/graph.hip).  capture_graph swaps it for a fill kernel:
    memset(buf, 0) -> buf += 1 must leave all ones after every replay."""
    import ctypes

    from monocular_depth_estimation_amd import _abi
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipMemsetAsync.restype = ctypes.c_int
    for n in (4, 4096, 1 << 20):
        buf = torch.zeros(n, dtype=torch.int32, device=DEV)
        s = torch.cuda.Stream()

        def body():
            assert hip.hipMemsetAsync(buf.data_ptr(), 0, n * 4, s.cuda_stream) == 0
            buf.add_(1)

        g, _, replaced = _abi.capture_graph(body, s)
        assert replaced == 1
        for _ in range(4):
            g.replay()
            torch.cuda.synchronize()
            assert int(buf.min()) == 1 and int(buf.max()) == 1


@pytest.mark.parametrize("rows,cin,cout", [(4800, 1024, 4096), (76800, 256, 1024)])
def test_bf16_linear_bias_grad_replays(rows, cin, cout):
    """The captured bf16-autocast Linear backward (NewCRF qk / fc1 shapes) gives
    the eager bias gradient on every replay (it did on the first replay only
    before the memset repair: ATen's multi-block column sum)."""
    from monocular_depth_estimation_amd import _abi
    torch.manual_seed(0)
    lin = torch.nn.Linear(cin, cout).to(DEV)
    x = torch.randn(1, rows, cin, device=DEV)
    go = torch.randn(1, rows, cout, device=DEV)

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            y = lin(x)
        y.backward(go.to(y.dtype))

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        lin.zero_grad(set_to_none=True)
        run()
    torch.cuda.current_stream().wait_stream(s)
    ref = lin.bias.grad.clone()
    lin.zero_grad(set_to_none=True)
    g, _, _ = _abi.capture_graph(run, s)
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(lin.bias.grad).all()
        assert float((lin.bias.grad - ref).abs().max()) <= 1e-6 * float(ref.abs().max())


def test_bf16_autocast_step_ptmodel():
    """cfg4 model under bf16 autocast: 3 graph replays == eager steps (the
    NewCRF Linear-bias gradients went non-finite from the 2nd replay before
    the memset repair).  256x320 bs 2: 10240 tokens at crf0."""
    from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
    le, _, pe = _run(PTModel, graph=False, amp="bf16", h=256, w=320)
    lg, moved, pg = _run(PTModel, graph=True, amp="bf16", h=256, w=320)
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-5 * abs(b), (lg, le)
    assert all(bool(torch.isfinite(p).all()) for p in pg.values())
    worst = max(float((pg[n] - pe[n]).abs().max()) for n in pe)
    assert worst <= 1e-5, worst
    assert min(moved) > 0.5e-4, moved


def test_bucketed_overlapped_allreduce_graph_matches_eager():
    """The N > 1 GraphTrainer path: gradients as views of bucket buffers, each
    bucket all-reduced (AVG) over RCCL on a side stream from a post-accumulate
    hook, captured INTO the step graph.  Run with a one-rank "nccl" group: the
    collectives are issued (GradBuckets issues them whenever buckets exist)
    and the average over one rank is the identity, so the replayed step must
    equal the eager Trainer to 1e-6.  The graph census proves the capture: the
    step graph has exactly one collective's worth of nodes per bucket more
    than the same step captured with the collective stubbed out.  Every
    parameter sits in exactly one bucket and the buckets stay the .grad
    storage across replays."""
    import os

    import torch.distributed as dist

    from monocular_depth_estimation_amd import GuideDepth, _abi
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, World, synthetic_batch
    own = not dist.is_initialized()
    if own:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    try:
        ref_losses, _, ref_params = _run(lambda: GuideDepth(pretrained=False), graph=False)
        # nodes one captured all_reduce(AVG) contributes
        probe = torch.ones(1 << 20, device=DEV)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_reduce(probe, op=dist.ReduceOp.AVG)  # eager warm-up of the communicator
        torch.cuda.synchronize()
        g1, _, _ = _abi.capture_graph(lambda: dist.all_reduce(probe, op=dist.ReduceOp.AVG), s)
        per_collective = g1.node_counts["total"]
        assert per_collective >= 1, g1.node_counts
        g1.replay()
        torch.cuda.synchronize()
        assert float(probe.min()) == 1.0 and float(probe.max()) == 1.0

        torch.manual_seed(0)
        model = GuideDepth(pretrained=False).to(DEV)
        world = World(0, 0, 1, torch.device(DEV))
        tr = GraphTrainer(model, SSIML1(1.0, 0.1, depth_norm=True), world, lr=1e-4,
                          dp_overlap=True)
        assert tr.buckets is not None and len(tr.buckets) >= 2
        seen = [p for ps, _ in tr.buckets for p in ps]
        assert len(seen) == len(tr.params) and len({id(p) for p in seen}) == len(seen)
        tr.begin_epoch()
        losses = []
        for k in range(6):
            image, depth = synthetic_batch(2, 64, 96, 0, k, DEV)
            losses.append(float(tr.step(image, depth).detach()))
        torch.cuda.synchronize()
        assert tr.graphs is not None and tr.graphs[1] is None  # one graph, collectives inside
        assert sorted(tr.buckets.launched) == list(range(len(tr.buckets)))
        for ps, flat in tr.buckets:  # .grad is still the bucket storage
            for p in ps:
                assert p.grad.data_ptr() >= flat.data_ptr()
                assert p.grad.data_ptr() < flat.data_ptr() + flat.numel() * flat.element_size()
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) <= 1e-6 * max(1.0, abs(b))
        for n, p in model.named_parameters():
            err = float((p.detach() - ref_params[n]).abs().max())
            assert err <= 1e-6 * max(1.0, float(ref_params[n].abs().max())), n
        with_coll = tr.graphs[0].node_counts
        tr.buckets._collective = lambda flat: None  # same step, collectives stubbed out
        tr.graphs = None
        tr._capture()
        without = tr.graphs[0].node_counts
        extra = with_coll["total"] - without["total"]
        assert extra == len(tr.buckets) * per_collective, (with_coll, without, per_collective,
                                                            len(tr.buckets))
    finally:
        if own:
            dist.destroy_process_group()
