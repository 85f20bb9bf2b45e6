"""Per-shape timing of the bf16 convolutions of DDRNet-23-slim at cfg3 sizes (bs 32):
convbf.hip (forward / data gradient / weight gradient, pack included) against
MIOpen's bf16 solvers (what autocast runs: F.conv2d / convolution_backward on
bf16 NCHW tensors, NHWC transposes included).  HIP events, median of 20.

    python tools/convbf_bench.py [--n 32] [--only 64,64,60,80,3,1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [
    (32, 32, 240, 320, 3, 2), (32, 64, 120, 160, 3, 2), (32, 64, 120, 160, 1, 2),
    (64, 64, 60, 80, 3, 1), (64, 128, 60, 80, 3, 2), (64, 64, 60, 80, 1, 1),
    (64, 128, 60, 80, 1, 1), (128, 64, 60, 80, 3, 1), (128, 128, 30, 40, 3, 1),
    (128, 256, 30, 40, 3, 2), (128, 64, 30, 40, 1, 1), (256, 256, 15, 20, 3, 1),
    (256, 256, 15, 20, 3, 2), (256, 64, 15, 20, 1, 1), (256, 512, 15, 20, 1, 2),
    (256, 256, 15, 20, 1, 1), (512, 128, 8, 10, 1, 1), (128, 128, 8, 10, 3, 1),
    (640, 256, 8, 10, 1, 1),
]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=32)
    p.add_argument("--only", default="")
    args = p.parse_args()
    from monocular_depth_estimation_amd import _abi
    shapes = [tuple(int(v) for v in args.only.split(","))] if args.only else SHAPES
    n = args.n
    tot = {"hip": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0]}
    print(f"{'shape (cin,cout,h,w,k,s)':30s} {'fwd hip/miopen us':>20s} {'dgrad':>16s} {'wgrad':>16s}"
          f"  fwd TF")
    for cin, cout, h, w, k, s in shapes:
        pad = k // 2
        ho, wo = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
        x = torch.randn((n, cin, h, w), device="cuda").to(torch.bfloat16)
        gy = torch.randn((n, cout, ho, wo), device="cuda").to(torch.bfloat16)
        wt = torch.randn((cout, cin, k, k), device="cuda") * 0.05
        wb = wt.to(torch.bfloat16)
        ok = [_abi.query("mde_convbf_supported", cin, cout, h, w, k, s, q) for q in (0, 1, 2)]
        st = _abi.stream_of(x)
        wp = torch.empty(_abi.query("mde_convbf_pack_elems", cin, cout, k, 0), dtype=torch.bfloat16,
                         device="cuda")
        wtp = torch.empty(_abi.query("mde_convbf_pack_elems", cin, cout, k, 1), dtype=torch.bfloat16,
                          device="cuda")
        y = torch.empty((n, cout, ho, wo), dtype=torch.bfloat16, device="cuda")
        gx = torch.empty_like(x)
        gw = torch.empty_like(wt)
        nws = _abi.query("mde_convbf_wgrad_workspace", n, cin, cout, h, w, k, s)
        ws = torch.empty(max(nws, 16), dtype=torch.uint8, device="cuda")

        def hf():
            _abi.call("mde_convbf_pack", _abi.ptr(wt), _abi.ptr(wp), cin, cout, k, 0, st)
            _abi.call("mde_convbf_fwd", _abi.ptr(x), _abi.ptr(wp), _abi.ptr(y), None, n, cin, cout, h,
                      w, k, s, st)

        def hd():
            _abi.call("mde_convbf_pack", _abi.ptr(wt), _abi.ptr(wtp), cin, cout, k, 1, st)
            _abi.call("mde_convbf_bwd_data", _abi.ptr(gy), _abi.ptr(wtp), _abi.ptr(gx), n, cin, cout,
                      h, w, k, s, st)

        def hw():
            _abi.call("mde_convbf_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin, cout, h, w,
                      k, s, _abi.ptr(ws), st)

        def mf():
            torch.nn.functional.conv2d(x, wt.to(torch.bfloat16), None, s, pad)

        def md():
            torch.ops.aten.convolution_backward(gy, x, wb, None, (s, s), (pad, pad), (1, 1), False,
                                                (0, 0), 1, (True, False, False))

        def mw():
            torch.ops.aten.convolution_backward(gy, x, wb, None, (s, s), (pad, pad), (1, 1), False,
                                                (0, 0), 1, (False, True, False))[1].float()

        th = [timeit(f) if o else float("nan") for f, o in zip((hf, hd, hw), ok)]
        tm = [timeit(f) for f in (mf, md, mw)]
        for i in range(3):
            if ok[i]:
                tot["hip"][i] += th[i]
                tot["miopen"][i] += tm[i]
        flops = 2.0 * n * ho * wo * cout * cin * k * k
        print(f"{str((cin, cout, h, w, k, s)):30s} {th[0]:8.1f} / {tm[0]:8.1f}  {th[1]:7.1f} / {tm[1]:7.1f}"
              f"  {th[2]:7.1f} / {tm[2]:7.1f}  {flops / th[0] / 1e6 if ok[0] else 0:7.1f}", flush=True)
    print(f"sum (supported passes): hip fwd {tot['hip'][0]:.1f} dgrad {tot['hip'][1]:.1f} "
          f"wgrad {tot['hip'][2]:.1f} us; miopen fwd {tot['miopen'][0]:.1f} dgrad "
          f"{tot['miopen'][1]:.1f} wgrad {tot['miopen'][2]:.1f} us")


if __name__ == "__main__":
    main()
