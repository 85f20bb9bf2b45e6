"""The guide convs (3 input channels, modules.py:52-54) at cfg2 / cfg3 sizes
(bs 32): fp32 (mde_conv3x3_fwd) and the autocast bf16-output kernel
(mde_conv3x3_guide_bf16_fwd, with its statistics epilogue), HIP-graph replay
timing; --reps N: just N launches per shape (rocprofv3 --pmc passes)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from monocular_depth_estimation_amd import _abi

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kbench  # noqa: E402

SHAPES = [(16, 480, 640), (32, 240, 320), (64, 120, 160)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=0)
    ap.add_argument("--cin16", action="store_true", help="the 16 -> 16 full-resolution convs instead")
    a = ap.parse_args()
    n = 32
    kbench._STREAM = torch.cuda.Stream()
    with torch.cuda.stream(kbench._STREAM):
        for co, h, w in ([(16, 480, 640)] if a.cin16 else SHAPES):
            ci = 16 if a.cin16 else 3
            x = torch.rand((n, ci, h, w), device="cuda")
            wt = (torch.rand((co, ci, 3, 3), device="cuda") - 0.5) * 0.5
            y = torch.empty((n, co, h, w), device="cuda")
            yb = torch.empty((n, co, h, w), dtype=torch.bfloat16, device="cuda")
            nb = _abi.query("mde_conv3x3_guide_bf16_stats_blocks", n, co, h, w)
            stats = torch.empty((co, nb, 4), device="cuda")
            st = _abi.stream_of(x)
            f32 = lambda: _abi.call("mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, ci, co,
                                    h, w, 0, st)
            nbf = _abi.query("mde_conv3x3_stats_blocks", n, ci, co, h, w, 0)
            stf = torch.empty((co, nbf, 4), device="cuda")
            f32s = lambda: _abi.call("mde_conv3x3_fwd_stats", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y),
                                     _abi.ptr(stf), n, ci, co, h, w, 0, st)
            b16 = lambda: _abi.call("mde_conv3x3_guide_bf16_fwd", _abi.ptr(x), _abi.ptr(wt),
                                    _abi.ptr(yb), _abi.ptr(stats), n, co, h, w, st)
            f32d = lambda: _abi.call("mde_conv3x3_bwd_data", _abi.ptr(y), _abi.ptr(wt), _abi.ptr(x), n,
                                     ci, co, h, w, 0, st)
            runs = (("fp32", f32, 4), ("fp32+stats", f32s, 4), ("bf16+stats", b16, 2))
            if a.cin16:
                runs = runs[:2] + (("fp32 dgrad", f32d, 4),)
            for name, f, ob in runs:
                if a.reps:
                    for _ in range(a.reps):
                        f()
                    torch.cuda.synchronize()
                    continue
                us = kbench.timeit(f, 20) * 1e3
                byts = n * h * w * (ci * 4 + co * ob)
                print(f"guide {ci}->{co} {h}x{w} {name}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s",
                      flush=True)


if __name__ == "__main__":
    main()
