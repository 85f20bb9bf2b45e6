"""Compare one GraphTrainer eager step with one Trainer step (grads / params)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from monocular_depth_estimation_amd import GuideDepth
from monocular_depth_estimation_amd.loss import SSIML1
from monocular_depth_estimation_amd.train import GraphTrainer, Trainer, World, make_adam, synthetic_batch

DEV = "cuda"
torch.backends.cudnn.deterministic = True
world = World(0, 0, 1, torch.device(DEV))
res = {}
for mode in ("eager", "graph", "eager2"):
    torch.manual_seed(0)
    m = GuideDepth(pretrained=False).to(DEV)
    lf = SSIML1(1.0, 0.1, depth_norm=True)
    tr = GraphTrainer(m, lf, world) if mode == "graph" else Trainer(m, make_adam(m), lf, world, False)
    tr.begin_epoch()
    image, depth = synthetic_batch(2, 64, 96, 0, 0, DEV)
    l = tr.step(image, depth)
    torch.cuda.synchronize()
    res[mode] = (float(l), {n: p.detach().clone() for n, p in m.named_parameters()},
                 {n: (p.grad.detach().clone() if p.grad is not None else None) for n, p in m.named_parameters()})
le, pe, ge = res["eager"]
lg, pg, gg = res["graph"]
l2, p2, g2 = res["eager2"]
print("loss", le, lg, l2)
print("eager vs eager2 grad maxdiff", max(float((ge[n] - g2[n]).abs().max()) for n in ge if ge[n] is not None))
print("eager vs eager2 param maxdiff", max(float((pe[n] - p2[n]).abs().max()) for n in pe))
bad = []
for n in pe:
    dp = float((pe[n] - pg[n]).abs().max())
    gdiff = None if ge[n] is None else float((ge[n] - gg[n]).abs().max())
    if dp > 1e-7 or ge[n] is None:
        bad.append((n, dp, gdiff, None if ge[n] is None else float(ge[n].abs().max())))
print(len(bad), "params differ")
for b in bad[:30]:
    print(b)
