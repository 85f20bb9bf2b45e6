"""Conditioning of the 64x96 bs-2 GuideDepth golden step's gradient norms.

Median relative gradient-norm error vs the float64 oracle (encoder /
decoder parameters separately) for: HIP fp32, HIP fp32 with the input
perturbed by 2^-9 relative noise (a bf16 rounding), HIP bf16 (MFMA conv3x3),
HIP bf16 with MIOpen for every 3x3, and the CPU bf16 autocast oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import monocular_depth_estimation_amd as mde
from monocular_depth_estimation_amd import nn as mnn
from monocular_depth_estimation_amd.loss import SSIML1
from oracle import guidedepth as og
from oracle import ops as oops
from oracle.weights import fill_

g = np.load("tests/golden/golden_guidedepth.npz")
x, d = torch.from_numpy(g["x"]), torch.from_numpy(g["depth"])
truth = fill_(og.GuideDepth()).double().train()
oops.train_loss(truth(x.double()), d.double()).backward()
want = {k: float(p.grad.norm()) for k, p in truth.named_parameters()}
top = max(want.values())


def med(model):
    enc, dec = [], []
    for k, p in model.named_parameters():
        if want[k] <= 1e-6 * top:
            continue
        r = abs(float(p.grad.double().norm()) - want[k]) / want[k]
        (enc if k.startswith("feature_extractor") else dec).append(r)
    return f"enc med {np.median(enc):.3f} p90 {np.percentile(enc, 90):.3f}  " \
           f"dec med {np.median(dec):.3f} p90 {np.percentile(dec, 90):.3f}"


def gpu(bf16, xin, table=None):
    saved = dict(mnn.CONV3X3_HIP_BF16)
    if table is not None:
        mnn.CONV3X3_HIP_BF16.clear()
        mnn.CONV3X3_HIP_BF16.update(table)
    try:
        m = fill_(mde.GuideDepth(pretrained=False)).cuda().train()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16, cache_enabled=False):
            loss = SSIML1(1.0, 0.1)(m(xin.cuda()), d.cuda())
        loss.backward()
        return m
    finally:
        mnn.CONV3X3_HIP_BF16.clear()
        mnn.CONV3X3_HIP_BF16.update(saved)


torch.backends.cudnn.deterministic = True
print("HIP fp32            ", med(gpu(False, x)), flush=True)
gen = torch.Generator().manual_seed(5)
for s in range(8):
    xp = x * (1 + (torch.rand(x.shape, generator=gen) - 0.5) * 2 ** -8)
    print(f"HIP fp32 perturbed {s}", med(gpu(False, xp)), flush=True)
print("HIP bf16 (MFMA)     ", med(gpu(True, x)), flush=True)
print("HIP bf16 (MIOpen)   ", med(gpu(True, x, {})), flush=True)
cpu = fill_(og.GuideDepth()).train()
with torch.autocast("cpu", dtype=torch.bfloat16):
    cp = cpu(x)
oops.train_loss(cp.float(), d).backward()
print("CPU bf16 oracle     ", med(cpu), flush=True)
