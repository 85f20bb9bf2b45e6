"""GraphTrainer's data-parallel path (N > 1) on the one-GPU box: two ranks share
cuda:0 and talk gloo over GPU tensors (RCCL refuses two ranks on one device;
the all-reduce / broadcast calls are the same torch.distributed API).

Checks: parameters are bitwise identical on both ranks after 5 steps (2
eager, capture, 2 replays) although each rank initialised differently (rank
0's weights are broadcast, gradients all-reduced), and each rank's loss is
its own shard's loss (ranks see different data, so the losses differ).  BN
running statistics are rank-local between steps, as under DDP (broadcast
from rank 0 before every forward), so they are not compared.
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


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, init_world, synthetic_batch
    w = init_world(backend="gloo", use_gpu=True, device_index=0)
    torch.manual_seed(rank)  # different init per rank: the trainer must broadcast rank 0's
    model = GuideDepth(pretrained=False).to(w.device)
    tr = GraphTrainer(model, SSIML1(1.0, 0.1, depth_norm=True), w, lr=1e-4)
    tr.begin_epoch()
    losses = []
    for k in range(5):
        image, depth = synthetic_batch(2, 64, 96, rank, k, w.device)
        losses.append(float(tr.step(image, depth).detach()))
    torch.cuda.synchronize()
    state = {k: v.detach().cpu() for k, v in model.named_parameters()}
    torch.save({"losses": losses, "state": state}, os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(900)
def test_graph_trainer_two_ranks_stay_in_sync():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0, r1 = (torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2))
    for k, v in r0["state"].items():
        assert torch.equal(v, r1["state"][k]), k
    assert r0["losses"] != r1["losses"]
