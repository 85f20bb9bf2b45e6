"""bench.py's own N-rank launcher (verdict r4 #1), on the CPU.

`python bench.py --gpus N` outside a torchrun job must start the N ranks
itself (torch.distributed.run as a child process, before any GPU call) and
print rank 0's single JSON line with n_gpus taken from the process group.
`--device cpu` runs that launcher and the data-parallel exchange (gloo,
GradBuckets) on a plain-torch stand-in net; every rank must end with the same
parameters although each starts from its own random init and trains on its
own shard.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--steps", "3",
           "--warmup", "1", "--bs", "2", "--height", "32", "--width", "48", *extra]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "address already in use" in r.stderr.lower():
        # the launcher's free port (bound, released, then handed to the
        # rendezvous) was taken by another process in between: one retry
        r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only, one line
    return json.loads(lines[0]), r.stderr


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    out, err = _run("--gpus", str(n))
    assert "launching" in err and "torch.distributed.run" in err
    assert out["n_gpus"] == n
    assert out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["global_batch"] == 2 * n
    assert out["params_in_sync"] is True
    assert out["dp_exchange"] and "gradient buckets" in out["dp_exchange"]


@pytest.mark.timeout(300)
def test_bench_single_rank_needs_no_launcher():
    out, err = _run("--gpus", "1")
    assert "launching" not in err
    assert out["n_gpus"] == 1 and out["params_in_sync"] is None and out["dp_exchange"] is None
