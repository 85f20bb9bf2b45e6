"""Graph replay == eager at the bench shapes, default (non-deterministic) MIOpen solvers.

    python tools/graph_check.py [guidedepth|newcrf] [fp32|bf16] [steps]

Same init and batches; prints both loss sequences, the max relative loss
difference and the max parameter difference after `steps` steps (2 eager
warm-up + capture + replays), and how many memset nodes the capture repaired.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monocular_depth_estimation_amd.loss import SSIML1  # noqa: E402
from monocular_depth_estimation_amd.train import (GraphTrainer, Trainer, World,  # noqa: E402
                                                  make_adam, synthetic_batch)

which = sys.argv[1] if len(sys.argv) > 1 else "guidedepth"
amp = sys.argv[2] if len(sys.argv) > 2 else "fp32"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
bs = 32 if which == "guidedepth" else 16
world = World(0, 0, 1, torch.device("cuda"))


def build():
    torch.manual_seed(0)
    if which == "guidedepth":
        from monocular_depth_estimation_amd import GuideDepth
        return GuideDepth(pretrained=False).cuda()
    from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
    return PTModel().cuda()


batches = [synthetic_batch(bs, 480, 640, 0, k, "cuda") for k in range(2)]
out = {}
for graph in (False, True):
    model = build()
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    tr = (GraphTrainer(model, loss_fn, world, lr=1e-4, amp=amp) if graph else
          Trainer(model, make_adam(model, 1e-4), loss_fn, world, eval_quirk=False, amp=amp))
    tr.begin_epoch()
    losses = [float(tr.step(*batches[k % 2]).detach()) for k in range(steps)]
    torch.cuda.synchronize()
    out[graph] = (losses, {n: p.detach().clone() for n, p in model.named_parameters()},
                  getattr(tr, "memsets_replaced", None))
le, pe, _ = out[False]
lg, pg, nrep = out[True]
rel = max(abs(a - b) / abs(b) for a, b in zip(lg, le))
dp = max(float((pg[n] - pe[n]).abs().max()) for n in pe)
finite = all(bool(torch.isfinite(p).all()) for p in pg.values())
print(f"{which} {amp}: eager {le}\n  graph {lg}\n  max rel loss diff {rel:.3e}, max param diff "
      f"{dp:.3e}, finite {finite}, memset nodes replaced {nrep}", flush=True)
sys.exit(0 if finite and rel < 1e-3 else 1)
