"""Child process of tests/test_gpu_graph.py's RCCL cases (not collected by pytest).

One-rank "nccl" (RCCL) group on cuda:0; GraphTrainer with the data-parallel
exchange forced on (dp_collectives=True: the average over one rank is the
identity), GuideDepth 2x64x96, 6 steps (2 eager, capture, 3 replays), against
the eager Trainer under MIOpen's deterministic solvers.

  flat     graph A (forward, backward, flat pack + 1/N) -> one EAGER RCCL
           all_reduce -> graph B (unpack, Adam): the N > 1 default;
  overlap  per-bucket all_reduce(AVG) on a side stream captured INTO the step
           graph (opt-in: MDE_DP_OVERLAP=1), plus the node census: exactly
           one collective's worth of nodes per bucket.

Runs in its own process so that a runtime abort (SIGABRT) cannot take the
test session down with it.  Exit 0 = every assertion held.
"""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

DEV = "cuda"


def _run(tr_factory, steps=6):
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.train import synthetic_batch
    torch.manual_seed(0)
    model = GuideDepth(pretrained=False).to(DEV)
    tr = tr_factory(model)
    tr.begin_epoch()
    losses = []
    for k in range(steps):
        image, depth = synthetic_batch(2, 64, 96, 0, k, DEV)
        losses.append(float(tr.step(image, depth).detach()))
        if os.environ.get("MDE_RCCL_TRACE"):
            print(f"  {type(tr).__name__} step {k} done", flush=True)
    torch.cuda.synchronize()
    return tr, model, losses


def main(mode):
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, Trainer, World, make_adam
    torch.backends.cudnn.deterministic = True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    world = World(0, 0, 1, torch.device(DEV))
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    _, ref_model, ref_losses = _run(lambda m: Trainer(m, make_adam(m, 1e-4), loss_fn, world,
                                                      eval_quirk=False))
    ref_params = {n: p.detach().clone() for n, p in ref_model.named_parameters()}
    per_collective = None
    if mode == "overlap":  # nodes one captured all_reduce(AVG) contributes
        probe = torch.ones(1 << 20, device=DEV)
        s_eager, s = torch.cuda.Stream(), torch.cuda.Stream()
        s_eager.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_eager):
            dist.all_reduce(probe, op=dist.ReduceOp.AVG)  # eager warm-up of the communicator
        torch.cuda.synchronize()
        # The eager collective's Work is still on the watchdog's list and its
        # completion event was recorded on s_eager.  The capture stays open
        # 0.35 s, so the watchdog (100 ms poll) queries that event while the
        # capture runs: legal because the capture is thread-local (a global
        # one forbids the query) and s_eager never joins it (an event last
        # recorded on a capturing stream cannot be queried) -- GraphTrainer's
        # stream rules (train.py)
        assert _abi.default_capture_mode() == "thread_local"

        def probe_step():
            time.sleep(0.35)
            dist.all_reduce(probe, op=dist.ReduceOp.AVG)

        s.wait_stream(torch.cuda.current_stream())
        g1, _, _ = _abi.capture_graph(probe_step, s)
        per_collective = g1.node_counts["total"]
        print(f"probe collective nodes: {g1.node_types}", flush=True)
        assert per_collective >= 1, g1.node_counts
        g1.replay()
        torch.cuda.synchronize()
        assert float(probe.min()) == 1.0 and float(probe.max()) == 1.0
        g1.reset()
    print(f"{mode}: eager reference done, graph trainer next", flush=True)
    tr, model, losses = _run(lambda m: GraphTrainer(
        m, loss_fn, world, lr=1e-4, dp_overlap=(mode == "overlap"), dp_collectives=True))
    ga, gb, _ = tr.graphs["train"]  # BN stays in train mode: the one captured step
    print(f"{mode}: step graph nodes: {[g.node_types for g in (ga, gb) if g is not None]}",
          flush=True)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(b)), (losses, ref_losses)
    for n, p in model.named_parameters():
        err = float((p.detach() - ref_params[n]).abs().max())
        assert err <= 1e-6 * max(1.0, float(ref_params[n].abs().max())), (n, err)
    if mode == "flat":
        assert tr.buckets is None and gb is not None  # two graphs, RCCL between
        assert tr.flat_grad is not None
        assert 0 < tr.flat_grad.numel() <= sum(p.numel() for p in tr.params)
    else:
        assert tr.buckets is not None and len(tr.buckets) >= 2
        seen = [p for ps, _ in tr.buckets for p in ps]
        assert len(seen) == len(tr.params) and len({id(p) for p in seen}) == len(seen)
        assert gb is None  # one graph, collectives inside
        assert sorted(tr.buckets.launched) == list(range(len(tr.buckets)))
        for ps, flat in tr.buckets:  # .grad is still the bucket storage
            for p in ps:
                assert flat.data_ptr() <= p.grad.data_ptr() < \
                    flat.data_ptr() + flat.numel() * flat.element_size()
        with_coll = ga.node_counts
        tr.close()
        tr.buckets._collective = lambda flat: None  # same step, collectives stubbed out
        tr.graphs["train"] = tr._capture()
        without = tr.graphs["train"][0].node_counts
        extra = with_coll["total"] - without["total"]
        assert extra == len(tr.buckets) * per_collective, (with_coll, without, per_collective)
    tr.close()
    del tr
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(f"OK {mode}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
