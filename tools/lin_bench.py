"""Linear weight gradients of the cfg4 step (NewCRF, bs 16): hipBLASLt's
g.t() @ x vs mde_linear_wgrad (+ the bias gradient), per shape, TF/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

# (tokens, M = out features, N = in features): qk, proj, fc1, fc2 at 1/4 .. 1/32
SHAPES = [(307200, 256, 128), (307200, 128, 128), (307200, 512, 128), (307200, 128, 512),
          (76800, 512, 256), (76800, 256, 256), (76800, 1024, 256), (76800, 256, 1024),
          (19200, 1024, 512), (19200, 512, 512), (19200, 2048, 512), (19200, 512, 2048),
          (4800, 2048, 1024), (4800, 1024, 1024), (4800, 4096, 1024), (4800, 1024, 4096)]


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
    return a.elapsed_time(b) / reps


def main():
    from monocular_depth_estimation_amd import _abi
    tot_b = tot_h = 0.0
    for t, m, n in SHAPES:
        g = torch.randn((t, m), device="cuda")
        x = torch.randn((t, n), device="cuda")
        gw = torch.empty((m, n), device="cuda")
        gb = torch.empty((m,), device="cuda")
        ws = torch.empty(_abi.query("mde_linear_wgrad_workspace", t, m, n) // 4, device="cuda")
        st = _abi.stream_of(g)
        tb = timeit(lambda: g.t() @ x)
        th = timeit(lambda: _abi.call("mde_linear_wgrad", _abi.ptr(g), _abi.ptr(x), _abi.ptr(gw),
                                      _abi.ptr(gb), t, m, n, _abi.ptr(ws), 0, st))
        fl = 2.0 * t * m * n
        tot_b += tb
        tot_h += th
        print(f"wgrad T={t:6d} M={m:4d} N={n:4d}: hipBLASLt {tb * 1e3:7.1f} us ({fl / tb / 1e9:6.1f} TF/s)"
              f"  hip {th * 1e3:7.1f} us ({fl / th / 1e9:6.1f} TF/s)", flush=True)
        del g, x, gw, gb, ws
    print(f"total: hipBLASLt {tot_b:.3f} ms, hip {tot_h:.3f} ms (one pass of each shape)")


if __name__ == "__main__":
    main()
