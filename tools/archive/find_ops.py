"""Where the step's ATen (non-HIP-kernel) ops come from: one eager GuideDepth
train step under torch.profiler with Python stacks; prints the top call
sites of fill / add / relu / copy ops.

    python tools/find_ops.py [--amp bf16] [--bs 32]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--amp", default="bf16")
    p.add_argument("--bs", type=int, default=32)
    a = p.parse_args()
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import GraphTrainer, init_world, synthetic_batch
    world = init_world(use_gpu=True)
    torch.manual_seed(0)
    model = GuideDepth(pretrained=False).to(world.device)
    tr = GraphTrainer(model, SSIML1(1.0, 0.1, depth_norm=True), world, lr=1e-4, amp=a.amp)
    img, dep = synthetic_batch(a.bs, 480, 640, 0, 0, world.device)
    tr.step(img, dep)  # eager (the first eager_steps calls are)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        tr.step(img, dep)
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::relu", "aten::clamp_min",
            "aten::threshold_backward", "aten::copy_", "aten::_to_copy", "aten::zeros", "aten::zeros_like")
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in want:
            st = [s for s in (ev.stack or []) if "monocular_depth_estimation_amd" in s or "torch/autograd" in s]
            key = (ev.name, str(ev.input_shapes)[:60], " <- ".join(s.split("/")[-1] for s in st[:3]))
            sites[key] += 1
    for (name, shp, st), c in sorted(sites.items(), key=lambda kv: -kv[1])[:60]:
        print(f"{c:4d} {name:28s} {shp:60s} {st}")


if __name__ == "__main__":
    main()
