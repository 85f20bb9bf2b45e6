"""Weight-gradient passes (MFMA partials + fixed-order reduction) of every
HIP 3x3 weight gradient in the cfg2 step (bs 32), timed per shape by HIP-graph
replays (kbench.timeit).  Run twice, MDE_WRED_SLICES=1 (one reduction launch)
vs default (sliced two-launch reduction where the partial rows are many)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from monocular_depth_estimation_amd import _abi
from monocular_depth_estimation_amd.nn import _ws

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kbench  # noqa: E402

# (cin, cout, h, w, stride, uses per cfg2 step)
SHAPES = [(3, 16, 480, 640, 1, 1), (16, 16, 480, 640, 1, 2), (3, 32, 240, 320, 1, 1),
          (32, 32, 240, 320, 1, 2), (3, 64, 120, 160, 1, 1), (32, 32, 120, 160, 1, 4),
          (64, 64, 60, 80, 1, 12), (64, 64, 120, 160, 1, 1), (128, 128, 30, 40, 1, 3),
          (256, 256, 15, 20, 1, 3), (128, 128, 8, 10, 1, 4),
          (3, 32, 480, 640, 2, 1), (32, 32, 240, 320, 2, 1), (32, 64, 120, 160, 2, 1),
          (64, 128, 60, 80, 2, 3), (128, 256, 30, 40, 2, 2)]


def main():
    kbench._STREAM = torch.cuda.Stream()
    n = 32
    tot = 0.0
    with torch.cuda.stream(kbench._STREAM):
        for ci, co, h, w, s, uses in SHAPES:
            ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
            x = torch.rand((n, ci, h, w), device="cuda") - 0.5
            gy = torch.rand((n, co, ho, wo), device="cuda") - 0.5
            gw = torch.empty((co, ci, 3, 3), device="cuda")
            st = _abi.stream_of(x)
            if s == 1:
                if not _abi.query("mde_conv3x3_supported", ci, co, 2, 0):
                    continue
                nws = _abi.query("mde_conv3x3_wgrad_workspace", n, ci, co, h, w, 0)
                fn = lambda: _abi.call("mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw),
                                       n, ci, co, h, w, _abi.ptr(ws), 0, st)
            else:
                nws = _abi.query("mde_conv3x3s2_wgrad_workspace", n, ci, co, h, w, 0)
                if nws <= 0:
                    continue
                fn = lambda: _abi.call("mde_conv3x3s2_wgrad", _abi.ptr(gy), _abi.ptr(x),
                                       _abi.ptr(gw), n, ci, co, h, w, _abi.ptr(ws), 0, st)
            ws = _ws(nws, x)
            us = kbench.timeit(fn, 20) * 1e3
            ref = torch.ops.aten.convolution_backward(gy, x, gw, None, (s, s), (1, 1), (1, 1), False,
                                                      (0, 0), 1, (False, True, False))[1]
            fn()
            err = float((gw - ref).abs().max() / ref.abs().max())
            tot += uses * us
            print(f"wgrad {ci}->{co} s{s} {h}x{w}: {us:7.1f} us  slab {nws / 1e6:6.1f} MB  "
                  f"rel diff {err:.1e}", flush=True)
    print(f"wgrad per cfg2 step (x uses): {tot:.0f} us  (MDE_WRED_SLICES="
          f"{os.environ.get('MDE_WRED_SLICES', 'auto')})", flush=True)


if __name__ == "__main__":
    main()
