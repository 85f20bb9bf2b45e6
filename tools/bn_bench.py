"""BatchNorm pass timings at the cfg2 shapes (bs 32): statistics (fwd_coef),
stats + apply (fwd_train), reduce + apply (bwd), apply alone (bwd_apply).

COLD=1: a 1 GiB scratch write before every timed call (evicts L2 / MALL, as
in the train step where the DDRNet convolutions run between the BN passes);
each call is timed alone with events.  SHAPES="c,h,w;..." overrides the list.
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from monocular_depth_estimation_amd import _abi  # noqa: E402

SHAPES = [(16, 240, 320), (32, 120, 160), (64, 60, 80), (8, 480, 640), (32, 240, 320), (128, 30, 40)]


COLD = os.environ.get("COLD") == "1"
_SCRATCH = []


def t(fn, reps=20):
    for _ in range(3):
        fn()
    if COLD:
        if not _SCRATCH:
            _SCRATCH.append(torch.empty(1 << 28, device="cuda"))
        tot = 0.0
        for _ in range(reps):
            _SCRATCH[0].fill_(1.0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            tot += a.elapsed_time(b)
        return tot * 1e3 / reps
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    n = 32
    f = dict(device="cuda", dtype=torch.float32)
    shapes = SHAPES
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in e.split(",")) for e in os.environ["SHAPES"].split(";")]
    for c, h, w in shapes:
        x = torch.randn((n, c, h, w), **f)
        gy = torch.randn_like(x)
        y, gx = torch.empty_like(x), torch.empty_like(x)
        g, b = torch.ones(c, **f), torch.zeros(c, **f)
        m, iv, sc, sh = (torch.empty(c, **f) for _ in range(4))
        gg, gb = torch.empty(c, **f), torch.empty(c, **f)
        sums = torch.zeros((c, 2), **f)
        ws = torch.empty(_abi.query("mde_batchnorm_workspace", n, c, h, w) // 4 + 1, **f)
        st = _abi.stream_of(x)
        P = _abi.ptr
        coef = lambda: _abi.call("mde_batchnorm_fwd_coef", P(x), P(g), P(b), None, None, None,  # noqa: E731
                                 None, 0.1, 1e-5, 1, P(sc), P(sh), P(m), P(iv), n, c, h, w, P(ws), 0, st)
        fwd = lambda: _abi.call("mde_batchnorm_fwd_train", P(x), P(g), P(b), None, None, None,  # noqa: E731
                                None, 0.1, 1e-5, None, P(y), P(m), P(iv), n, c, h, w, 1, P(ws), 0, st)
        bwd = lambda: _abi.call("mde_batchnorm_bwd", P(gy), P(x), None, P(g), P(b), P(m), P(iv), 1,  # noqa: E731
                                P(gx), None, P(gg), P(gb), None, n, c, h, w, 1, P(ws), 0, st)
        app = lambda: _abi.call("mde_batchnorm_bwd_apply", P(gy), P(x), None, P(g), P(b), P(m),  # noqa: E731
                                P(iv), 1, P(sums), P(gx), None, P(gg), P(gb), None, n, c, h, w, 1, 0, st)
        mb = 4.0 * x.numel() / 1e6
        tc, tf, tb, ta = t(coef), t(fwd), t(bwd), t(app)
        print(f"c{c:4d} {h}x{w}: tensor {mb:7.1f} MB | stats {tc:7.1f} us ({mb / tc:5.2f} TB/s) | "
              f"apply {tf - tc:7.1f} us ({2 * mb / (tf - tc):5.2f}) | reduce {tb - ta:7.1f} us "
              f"({2 * mb / (tb - ta):5.2f}) | bwd apply {ta:7.1f} us ({3 * mb / ta:5.2f})", flush=True)


if __name__ == "__main__":
    main()
