"""1x1 convolution backward at the DDRNet / DAPPM shapes of the cfg2 step
(bs 32): MIOpen (aten.convolution_backward, NHWC igemm + transposes) vs batched
GEMMs straight on NCHW (gx = W^T gy per image, gW = sum_n gy_n x_n^T)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

SHAPES = [(64, 128, 1, 60, 80), (64, 64, 1, 60, 80), (128, 64, 1, 30, 40), (256, 64, 1, 15, 20),
          (256, 256, 1, 15, 20), (256, 512, 1, 8, 10), (512, 128, 1, 8, 10), (640, 128, 1, 8, 10),
          (32, 64, 2, 120, 160), (64, 128, 2, 60, 80), (128, 256, 2, 30, 40), (256, 512, 2, 15, 20)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def gemm_bwd(gy, x, w, s):
    n, co = gy.shape[:2]
    xs = x[:, :, ::s, ::s] if s > 1 else x
    ci = x.shape[1]
    g3 = gy.reshape(n, co, -1)
    gw = torch.matmul(g3, xs.reshape(n, ci, -1).transpose(1, 2)).sum(0) if s == 1 else \
        torch.matmul(g3, xs.contiguous().reshape(n, ci, -1).transpose(1, 2)).sum(0)
    gxs = torch.matmul(w.reshape(co, ci).t(), g3).reshape(xs.shape)
    if s == 1:
        return gxs, gw
    gx = torch.zeros_like(x)
    gx[:, :, ::s, ::s] = gxs
    return gx, gw


for (ci, co, s, h, w) in SHAPES:
    n = 32
    x = torch.randn(n, ci, h, w, device="cuda")
    wt = torch.randn(co, ci, 1, 1, device="cuda") * 0.1
    gy = torch.randn(n, co, (h - 1) // s + 1, (w - 1) // s + 1, device="cuda")
    mio = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (s, s), (0, 0), (1, 1), False,
                                                      (0, 0), 1, (True, True, False))
    gem = lambda: gemm_bwd(gy, x, wt, s)
    tm, tg = timeit(mio), timeit(gem)
    a, b = mio(), gem()
    e1 = float((a[0] - b[0]).abs().max() / a[0].abs().max())
    e2 = float((a[1] - b[1].reshape(a[1].shape)).abs().max() / a[1].abs().max())
    print(f"1x1 {ci}->{co} s{s} {h}x{w}: MIOpen {tm:7.1f} us  GEMM {tg:7.1f} us  err {e1:.1e} {e2:.1e}",
          flush=True)
