"""Which vendor kernels MIOpen / rocBLAS run for each convolution of the cfg2
GuideDepth step that stays on ATen (fp32, bs 32): forward, data gradient and
weight gradient per shape, with device times (torch.profiler).  Shapes that
the HIP kernels take are listed for reference only."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

# (cin, cout, k, stride, H_in, W_in, count) of GuideDepth at 640x480 (tools: hooks on the oracle)
SHAPES = [(3, 32, 3, 2, 480, 640, 1), (32, 32, 3, 2, 240, 320, 1), (32, 64, 3, 2, 120, 160, 1),
          (64, 128, 3, 2, 60, 80, 3), (128, 256, 3, 2, 30, 40, 2), (256, 256, 3, 2, 15, 20, 1),
          (32, 64, 1, 2, 120, 160, 1), (64, 128, 1, 2, 60, 80, 1), (128, 256, 1, 2, 30, 40, 1),
          (256, 512, 1, 2, 15, 20, 1), (64, 128, 1, 1, 60, 80, 2), (64, 64, 1, 1, 60, 80, 2),
          (128, 64, 1, 1, 30, 40, 1), (256, 64, 1, 1, 15, 20, 1), (256, 256, 1, 1, 15, 20, 1),
          (256, 512, 1, 1, 8, 10, 1), (512, 128, 1, 1, 8, 10, 2), (640, 128, 1, 1, 8, 10, 1),
          (128, 128, 3, 1, 8, 10, 4), (64, 64, 1, 1, 120, 160, 1)]


def main():
    dev = torch.device("cuda")
    n = 32
    for (ci, co, k, s, h, w, cnt) in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev, requires_grad=True)
        wt = torch.randn(co, ci, k, k, device=dev, requires_grad=True)
        y = torch.nn.functional.conv2d(x, wt, None, s, k // 2)
        gy = torch.randn_like(y)
        mask = (ci != 3, True, False)  # the image needs no gradient
        bwd = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (s, s), (k // 2, k // 2),
                                                          (1, 1), False, (0, 0), 1, mask)
        for _ in range(3):  # solver selection / warm-up outside the profile
            torch.nn.functional.conv2d(x, wt, None, s, k // 2)
            bwd()
        torch.cuda.synchronize()
        res = {}
        for phase in ("fwd", "bwd"):
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                for _ in range(5):
                    if phase == "fwd":
                        torch.nn.functional.conv2d(x, wt, None, s, k // 2)
                    else:
                        bwd()
                torch.cuda.synchronize()
            agg = collections.defaultdict(float)
            for e in prof.events():
                if e.device_type.name == "CUDA":
                    agg[e.name[:60]] += e.device_time / 5
            res[phase] = agg
        tot = {p: sum(v.values()) for p, v in res.items()}
        print(f"== {ci}->{co} k{k} s{s} {h}x{w} (x{cnt}): fwd {tot['fwd']:.1f} us, bwd {tot['bwd']:.1f} us",
              flush=True)
        for p in ("fwd", "bwd"):
            for name, t in sorted(res[p].items(), key=lambda kv: -kv[1]):
                if t > 1.0:
                    print(f"     {p} {t:8.1f} us  {name}")


if __name__ == "__main__":
    main()
