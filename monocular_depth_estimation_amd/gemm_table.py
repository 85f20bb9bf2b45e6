"""Solution table for the vendor (hipBLASLt / rocBLAS) GEMMs left on the path.

The NewCRF / SAM Linears' forward and data-gradient GEMMs (and the few small
strided-batched ones) stay library GEMMs -- the weight gradients run on
mde_linear_wgrad (newcrf_layers.py).  PyTorch picks a hipBLASLt heuristic
solution per shape; PyTorch's TunableOp can instead time every hipBLASLt and
rocBLAS solution for a shape and keep the fastest.  `tunableop_gfx950.csv` is
that table for the bench workloads' shapes, made once on an MI355X of this
image (`tools/jobs/gpu_r06u.sh`: TunableOp tuning over cfg2 / cfg3 / cfg4 and
the SAM model, one run each); its validator lines pin PyTorch, HIP,
hipBLASLt, rocBLAS and the gfx950 target, and TunableOp ignores a table whose
validators do not match.  enable() loads it with tuning OFF: a listed shape
runs its recorded solution, any other shape the library default (no timing
at run time, nothing written).  MDE_GEMM_TABLE=0 leaves PyTorch's defaults.
"""
from __future__ import annotations

import os

import torch

TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")


def enable(path: str | None = None) -> str | None:
    """Load the solution table (tuning off); returns its path, or None when it
    is switched off, absent, or refused by TunableOp's validators."""
    path = path or TABLE
    if (os.environ.get("MDE_GEMM_TABLE", "1") == "0" or not torch.cuda.is_available()
            or not os.path.exists(path)):
        return None
    if os.environ.get("PYTORCH_TUNABLEOP_TUNING") == "1":
        return None  # a tuning run (tools/jobs) drives TunableOp through its own env
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    if not tun.read_file(path):
        tun.enable(False)
        return None
    return path
