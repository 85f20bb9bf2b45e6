"""Winograd F(2x2, 3x3) forward per shape (bs 32), HIP-graph replay timing
(kbench.timeit); with --reps N and no timing, just N launches per shape (for
rocprofv3 --pmc passes)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from monocular_depth_estimation_amd import _abi

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kbench  # noqa: E402

SHAPES = [(64, 64, 60, 80), (32, 32, 120, 160), (32, 32, 240, 320), (16, 16, 480, 640),
          (128, 128, 30, 40)]
# cfg4 (bs 16): the NewCRF projections' Winograd passes (forward cin -> cout,
# data gradient cout -> cin), newcrf_layers.py NewCRF.proj_x / proj_v
SHAPES_NC = [(160, 1024, 15, 20), (512, 1024, 15, 20), (1024, 512, 15, 20), (1024, 160, 15, 20),
             (112, 512, 30, 40), (256, 512, 30, 40), (512, 256, 30, 40), (128, 256, 60, 80),
             (64, 128, 120, 160)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=0)
    ap.add_argument("--only", default="", help="ci,co,h,w")
    ap.add_argument("--newcrf", action="store_true", help="cfg4's shapes at bs 16")
    ap.add_argument("--modes", default="1", help="mde_wino_mode values to time, e.g. 0,1")
    a = ap.parse_args()
    shapes = SHAPES_NC if a.newcrf else SHAPES
    if a.only:
        shapes = [tuple(int(v) for v in a.only.split(","))]
    n = 16 if a.newcrf else 32
    kbench._STREAM = torch.cuda.Stream()
    with torch.cuda.stream(kbench._STREAM):
        for ci, co, h, w in shapes:
            x = torch.rand((n, ci, h, w), device="cuda") - 0.5
            wt = (torch.rand((co, ci, 3, 3), device="cuda") - 0.5) * 0.1
            y = torch.empty((n, co, h, w), device="cuda")
            u = torch.empty(_abi.query("mde_wino_weight_bytes", ci, co) // 4, device="cuda")
            st = _abi.stream_of(x)
            _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), ci, co, 0, st)
            f = lambda: _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(y), n, ci, co, h,
                                  w, 0, 0, st)
            for mode in (int(m) for m in a.modes.split(",")):
                _abi.query("mde_wino_mode", mode)
                if a.reps:
                    for _ in range(a.reps):
                        f()
                    torch.cuda.synchronize()
                    continue
                us = kbench.timeit(f, 20) * 1e3
                fl = 2.0 * 9 * n * h * w * ci * co
                print(f"wino mode {mode} {ci}->{co} {h}x{w}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s "
                      f"direct-equiv, {fl / 2.25 / us / 1e6:6.1f} TF/s MFMA "
                      f"({fl / 2.25 / us / 1e6 / 157.3:5.1%})", flush=True)


if __name__ == "__main__":
    main()
