"""bf16 pointwise (BN-ReLU-fused 1x1) backward at the decoder shapes, bs 32:
time and effective bandwidth of mde_pointwise_bwd_bn (cin <= 32) /
mde_pointwise_bwd, algorithmic bytes = gy + y1 read once + gz written.

    python tools/pw_bf16_bench.py [--only 16,8,480,640] [--dtype bf16|fp32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(16, 8, 480, 640), (32, 16, 240, 320), (64, 32, 120, 160), (16, 16, 480, 640),
          (32, 32, 240, 320), (64, 64, 120, 160)]


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
    p.add_argument("--only", default="")
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--n", type=int, default=32)
    a = p.parse_args()
    from monocular_depth_estimation_amd import _abi
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    code = _abi.MDE_BF16 if a.dtype == "bf16" else _abi.MDE_F32
    shapes = [tuple(int(v) for v in a.only.split(","))] if a.only else SHAPES
    n = a.n
    f32 = dict(device="cuda", dtype=torch.float32)
    for cin, cout, h, w in shapes:
        y1 = (torch.rand((n, cin, h, w), **f32) * 2 - 0.7).to(dt)
        gy = (torch.rand((n, cout, h, w), **f32) - 0.5).to(dt)
        w2 = torch.rand((cout, cin), **f32) - 0.5
        sc, sh, mean = torch.rand(cin, **f32) + 0.5, torch.rand(cin, **f32) - 0.5, torch.rand(cin, **f32)
        gz = torch.empty_like(y1)
        gw = torch.empty_like(w2)
        sums = torch.empty((cin, 2), **f32)
        ws = torch.empty(_abi.query("mde_pointwise_workspace", n, cin, cout, h, w) // 4 + 16, **f32)
        st = _abi.stream_of(y1)
        es = y1.element_size()
        nbytes = es * n * h * w * (cout + 2 * cin)
        if cin <= 32:
            fn = lambda: _abi.call("mde_pointwise_bwd_bn", _abi.ptr(gy), _abi.ptr(y1), _abi.ptr(sc),  # noqa: E731
                                   _abi.ptr(sh), _abi.ptr(mean), _abi.ptr(w2), _abi.ptr(gz),
                                   _abi.ptr(gw), _abi.ptr(sums), n, cin, cout, h, w, _abi.ptr(ws),
                                   code, st)
        else:
            fn = lambda: _abi.call("mde_pointwise_bwd", _abi.ptr(gy), _abi.ptr(y1), _abi.ptr(sc),  # noqa: E731
                                   _abi.ptr(sh), _abi.ptr(w2), _abi.ptr(gz), _abi.ptr(gw), n, cin,
                                   cout, h, w, _abi.ptr(ws), code, st)
        us = timeit(fn)
        print(f"pointwise_bwd {a.dtype} {cin}->{cout} @{h}x{w}: {us:8.1f} us  "
              f"{nbytes / us / 1e3:7.1f} GB/s", flush=True)
        y2 = torch.empty_like(gy)
        ff = lambda: _abi.call("mde_pointwise_fwd", _abi.ptr(y1), _abi.ptr(sc), _abi.ptr(sh),  # noqa: E731
                               _abi.ptr(w2), _abi.ptr(y2), n, cin, cout, h, w, code, st)
        us = timeit(ff)
        fb = es * n * h * w * (cout + cin)
        print(f"pointwise_fwd {a.dtype} {cin}->{cout} @{h}x{w}: {us:8.1f} us  "
              f"{fb / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
