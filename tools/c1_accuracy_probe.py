"""1x1 channel mix (mde_conv1x1_fwd / _bwd_data) error vs float64 on random
data: max and mean |err| / rms(ref), for A/B of kernel variants via env."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from monocular_depth_estimation_amd import _abi
    g = torch.Generator().manual_seed(0)
    for cin, cout, h, w in ((32, 16, 32, 48), (16, 16, 64, 96), (40, 120, 60, 80), (24, 72, 120, 160)):
        n = 4
        x = torch.rand((n, cin, h, w), generator=g) - 0.5
        wt = (torch.rand((cout, cin), generator=g) - 0.5) * 0.2
        gy = torch.rand((n, cout, h, w), generator=g) - 0.5
        yr = torch.einsum("oc,nchw->nohw", wt.double(), x.double())
        gxr = torch.einsum("oc,nohw->nchw", wt.double(), gy.double())
        xd, wd, gyd = x.cuda(), wt.cuda(), gy.cuda()
        y = torch.empty((n, cout, h, w), device="cuda")
        gx = torch.empty((n, cin, h, w), device="cuda")
        st = _abi.stream_of(xd)
        _abi.call("mde_conv1x1_fwd", _abi.ptr(xd), _abi.ptr(wd), _abi.ptr(y), n, cin, cout, h, w, 1,
                  0, st)
        _abi.call("mde_conv1x1_bwd_data", _abi.ptr(gyd), _abi.ptr(wd), _abi.ptr(gx), n, cin, cout, h,
                  w, 1, 0, st)
        torch.cuda.synchronize()
        f32 = torch.einsum("oc,nchw->nohw", wt, x)  # CPU fp32 (sequential-ish sums)
        for name, got, ref in (("fwd", y.cpu(), yr), ("dgrad", gx.cpu(), gxr), ("cpu-fp32 fwd", f32, yr)):
            e = (got.double() - ref).abs()
            rms = ref.pow(2).mean().sqrt()
            print(f"{cin:4d}->{cout:<4d} {h}x{w} {name:13s} max {float(e.max() / rms):.3e} "
                  f"mean {float(e.mean() / rms):.3e}  bias {float((got.double() - ref).mean() / rms):+.2e}")


if __name__ == "__main__":
    main()
