"""GraphTrainer's data-parallel path (N > 1) on the one-GPU box: two ranks share
cuda:0 and talk gloo over GPU tensors (RCCL refuses two ranks on one device;
the all-reduce / broadcast calls are the same torch.distributed API).

Two exchange schemes, both checked:
  flat     -- gloo's default in GraphTrainer: graph A -> one flat all-reduce
              -> graph B (2 eager steps, capture, 2 replays);
  buckets  -- the overlapped GradBuckets path bench.py runs over RCCL on 8
              GPUs (hook-driven per-bucket all-reduce on a side stream); gloo
              cannot be captured, so it runs the step eagerly (eager_steps).
Checks: (1) the FIRST step's averaged gradient on every rank equals the mean
of the two ranks' local gradients, snapshotted just before the exchange
(to 1e-6: the sum of two fp32 values); (1b) flat: the local gradient the
first REPLAYED step contributes equals an independent eager forward +
backward of a fresh model holding the same weights on the same shard (so a
wrong local gradient under capture -- stale packed filters, stale BN
statistics -- fails; 1e-5 of each tensor's scale under MIOpen's
deterministic solvers); (2) the
parameters are bitwise identical on both ranks after 5 steps although each
rank initialised differently (rank 0's weights are broadcast, gradients
averaged); (3) each rank's loss is its own shard's loss (the losses differ).
BN running statistics are rank-local between steps (GraphTrainer does not
broadcast them every step) and rank 0's reach every rank on sync_buffers().
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, mode):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.backends.cudnn.deterministic = True
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, init_world, synthetic_batch
    w = init_world(backend="gloo", use_gpu=True, device_index=0)
    torch.manual_seed(rank)  # different init per rank: the trainer must broadcast rank 0's
    model = GuideDepth(pretrained=False).to(w.device)
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    if mode == "buckets":
        tr = GraphTrainer(model, loss_fn, w, lr=1e-4, dp_overlap=True, eager_steps=1000)
        assert tr.buckets is not None and len(tr.buckets) >= 2
    else:
        tr = GraphTrainer(model, loss_fn, w, lr=1e-4)
        assert tr.buckets is None
    tr.begin_epoch()
    params = tr.params
    # each rank's LOCAL step-0 gradients, snapshotted just before the exchange
    # (flat: the packed buffer, already scaled by 1/N; buckets: each bucket
    # before its 1/N scale and all_reduce), so the averaged gradients can be
    # checked against exactly what the ranks contributed -- a recomputation
    # through autograd is no reference here: at 64x96, bs 2, DAPPM's 1x1
    # BatchNorms over two values amplify rounding differences into percents
    local = {}
    step = [0]
    if mode == "flat":
        orig = tr._allreduce

        def snap_allreduce():
            key = "flat" if step[0] == 0 else f"flat{step[0]}"
            if key not in local and tr.flat_grad is not None:
                local[key] = tr.flat_grad.detach().cpu().clone()
            orig()
        tr._allreduce = snap_allreduce
    else:
        origc = tr.buckets._collective
        ptrs = {f.data_ptr(): i for i, f in enumerate(tr.buckets.buffers)}

        def snap_collective(flat):
            key = f"bucket{ptrs[flat.data_ptr()]}"
            if key not in local:
                torch.cuda.current_stream().synchronize()
                local[key] = flat.detach().cpu().clone()
            origc(flat)
        tr.buckets._collective = snap_collective
    losses = []
    first = None
    avg = None
    replay_k = tr.eager_steps  # the first step that runs from the captured graph
    ref = None
    for k in range(5):
        step[0] = k
        image, depth = synthetic_batch(2, 64, 96, rank, k, w.device)
        if mode == "flat" and k == replay_k:  # the same weights, for the eager recomputation
            torch.cuda.synchronize()
            ref = GuideDepth(pretrained=False).to(w.device)
            ref.load_state_dict(model.state_dict())
            ref.train()
            ref_batch = (image.clone(), depth.clone())
        losses.append(float(tr.step(image, depth).detach()))
        if k == 0:
            torch.cuda.synchronize()
            first = [p.grad.detach().clone() for p in params]
            if mode == "buckets":
                avg = [f.detach().cpu().clone() for f in tr.buckets.buffers]
    torch.cuda.synchronize()
    eager = None
    if ref is not None:  # independent eager local gradient at the replayed step's weights
        ref.zero_grad(set_to_none=True)
        loss_fn(ref(ref_batch[0]), ref_batch[1]).backward()
        torch.cuda.synchronize()
        eager = [(p.grad.detach().cpu() / w.size) if p.grad is not None else torch.zeros_like(p).cpu()
                 for p in ref.parameters() if p.requires_grad]
    state = {k: v.detach().cpu() for k, v in model.named_parameters()}
    # BN running statistics: rank-local during training (no per-step
    # broadcast), rank 0's to every rank on sync_buffers()
    bn_local = tr.flat_bn.detach().cpu().clone()
    tr.sync_buffers()
    torch.cuda.synchronize()
    bn_synced = tr.flat_bn.detach().cpu().clone()
    tr.close()
    torch.save({"losses": losses, "state": state, "local": local, "avg": avg, "eager": eager,
                "replay_k": replay_k,
                "bn_local": bn_local, "bn_synced": bn_synced,
                "first": [g.cpu() for g in first]},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["flat", "buckets"])
def test_graph_trainer_two_ranks(mode):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, mode), nprocs=2, join=True)
        r0, r1 = (torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2))
    for a, b in zip(r0["first"], r1["first"]):  # one averaged gradient on both ranks
        assert torch.equal(a, b)
    # the averaged gradient is the mean of what the two ranks contributed
    l0, l1 = r0["local"], r1["local"]
    assert l0.keys() == l1.keys() and l0
    assert not all(torch.equal(l0[k], l1[k]) for k in l0)  # the shards differ
    if mode == "flat":
        want = (l0["flat"] + l1["flat"]).split([g.numel() for g in r0["first"]])
        got = r0["first"]
    else:
        assert len(l0) == len(r0["avg"])  # every bucket exchanged in step 0
        want = [0.5 * l0[f"bucket{i}"] + 0.5 * l1[f"bucket{i}"] for i in range(len(r0["avg"]))]
        got = r0["avg"]
    for g, m in zip(got, want):
        m = m.view_as(g)
        assert float((g - m).abs().max()) <= 1e-6 * float(m.abs().max()) + 1e-12
    if mode == "flat":  # (1b) the replayed step's local gradient vs an eager recomputation
        for r in (r0, r1):
            key = f"flat{r['replay_k']}"
            assert key in r["local"], sorted(r["local"])
            got = r["local"][key].split([g.numel() for g in r["eager"]])
            gmax = max(float(g.abs().max()) for g in r["eager"])
            worst = 0.0
            for g, e in zip(got, r["eager"]):
                scale = max(float(e.abs().max()), 1e-6 * gmax)
                worst = max(worst, float((g.view_as(e) - e).abs().max()) / scale)
            assert worst <= 1e-5, worst
    for k, v in r0["state"].items():
        assert torch.equal(v, r1["state"][k]), k
    assert r0["losses"] != r1["losses"]
    assert torch.equal(r0["bn_local"], r0["bn_synced"])  # rank 0 keeps its own statistics
    assert not torch.equal(r0["bn_local"], r1["bn_local"])  # per-shard batch statistics
    assert torch.equal(r1["bn_synced"], r0["bn_local"])  # rank 0's, on every rank
