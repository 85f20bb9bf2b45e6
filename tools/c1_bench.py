"""DDRNet's wide 1x1 convolutions at cfg2 (bs 32): the NCHW HIP kernels
(mde_conv1x1_fwd / _bwd_data / _wgrad incl. its reduction) vs MIOpen
(F.conv2d / aten.convolution_backward on NCHW tensors, incl. its layout
transposes).  Times from HIP-graph replays (kbench.timeit)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from monocular_depth_estimation_amd import _abi
from monocular_depth_estimation_amd.nn import _ws

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kbench  # noqa: E402

# (cin, cout, stride, h, w, uses per cfg2 step)
SHAPES = [(32, 64, 2, 120, 160, 1), (64, 128, 2, 60, 80, 1), (128, 256, 2, 30, 40, 1),
          (256, 512, 2, 15, 20, 1), (64, 128, 1, 60, 80, 2), (128, 64, 1, 30, 40, 1),
          (256, 64, 1, 15, 20, 1), (256, 256, 1, 15, 20, 1), (256, 512, 1, 8, 10, 1),
          (512, 128, 1, 8, 10, 2), (640, 128, 1, 8, 10, 1)]

# (cin, cout, h, w, uses per cfg2 step) of the stride-2 3x3 convs (input sizes)
S2_SHAPES = [(3, 32, 480, 640, 1), (32, 32, 240, 320, 1), (32, 64, 120, 160, 1), (64, 128, 60, 80, 3),
             (128, 256, 30, 40, 2), (256, 256, 15, 20, 1)]
# stride-1 3x3 on the wide kernel (BasicBlocks, DAPPM process, head): (cin, cout, h, w, uses)
S1_SHAPES = [(32, 32, 120, 160, 4), (64, 64, 60, 80, 12), (128, 128, 30, 40, 3),
             (256, 256, 15, 20, 3), (128, 128, 8, 10, 4), (128, 64, 60, 80, 1)]


def main():
    kbench._STREAM = torch.cuda.Stream()
    with torch.cuda.stream(kbench._STREAM):
        run()


def run():
    n = 32
    tot = {"hip": 0.0, "miopen": 0.0}
    for ci, co, s, h, w, uses in SHAPES:
        ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
        x = torch.rand((n, ci, h, w), device="cuda") - 0.5
        wt = (torch.rand((co, ci, 1, 1), device="cuda") - 0.5) * 0.1
        gy = torch.rand((n, co, ho, wo), device="cuda") - 0.5
        y = torch.empty_like(gy)
        gx = torch.empty_like(x)
        gw = torch.empty_like(wt)
        ws = _ws(_abi.query("mde_conv1x1_wgrad_workspace", n, ci, co, h, w, s, 0), x)
        st = _abi.stream_of(x)
        fwd = lambda: _abi.call("mde_conv1x1_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, ci, co,
                                h, w, s, 0, st)
        dgr = lambda: _abi.call("mde_conv1x1_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n,
                                ci, co, h, w, s, 0, st)
        wgr = lambda: _abi.call("mde_conv1x1_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, ci,
                                co, h, w, s, _abi.ptr(ws), 0, st)
        mf = lambda: torch.nn.functional.conv2d(x, wt, None, s)
        mb = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (s, s), (0, 0), (1, 1),
                                                         False, (0, 0), 1, (True, True, False))
        t = {k: kbench.timeit(f, 20) * 1e3 for k, f in
             (("fwd", fwd), ("dgrad", dgr), ("wgrad", wgr), ("mio_fwd", mf), ("mio_bwd", mb))}
        fl = 2.0 * n * ho * wo * ci * co
        mgx, mgw = mb()[:2]
        fwd()
        dgr()
        wgr()
        ym = mf()
        err = max(float((a - b).abs().max() / b.abs().max()) for a, b in
                  ((y, ym), (gx, mgx), (gw, mgw)))
        hip = t["fwd"] + t["dgrad"] + t["wgrad"]
        mio = t["mio_fwd"] + t["mio_bwd"]
        tot["hip"] += uses * hip
        tot["miopen"] += uses * mio
        print(f"1x1 {ci}->{co} s{s} {h}x{w}: HIP fwd {t['fwd']:6.1f} dgrad {t['dgrad']:6.1f} "
              f"wgrad {t['wgrad']:6.1f} us ({fl / t['fwd'] / 1e6:5.1f} / {fl / t['dgrad'] / 1e6:5.1f} / "
              f"{fl / t['wgrad'] / 1e6:5.1f} TF/s) | MIOpen fwd {t['mio_fwd']:6.1f} bwd {t['mio_bwd']:6.1f} us"
              f" | rel diff {err:.1e}", flush=True)
    print(f"1x1 per cfg2 step (x uses): HIP {tot['hip']:.0f} us, MIOpen {tot['miopen']:.0f} us",
          flush=True)
    # stride-2 3x3 (forward + data gradient; the weight gradient was already on HIP)
    tot = {"hip": 0.0, "miopen": 0.0}
    for ci, co, h, w, uses in S2_SHAPES:
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        x = torch.rand((n, ci, h, w), device="cuda") - 0.5
        wt = (torch.rand((co, ci, 3, 3), device="cuda") - 0.5) * 0.1
        gy = torch.rand((n, co, ho, wo), device="cuda") - 0.5
        y = torch.empty_like(gy)
        gx = torch.empty_like(x)
        st = _abi.stream_of(x)
        fwd = lambda: _abi.call("mde_conv3x3s2_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, ci, co,
                                h, w, 0, st)
        dgr = lambda: _abi.call("mde_conv3x3s2_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n,
                                ci, co, h, w, 0, st)
        mf = lambda: torch.nn.functional.conv2d(x, wt, None, 2, 1)
        md = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (2, 2), (1, 1), (1, 1),
                                                         False, (0, 0), 1, (True, False, False))
        passes = (("fwd", fwd), ("mio_fwd", mf)) if ci == 3 else \
            (("fwd", fwd), ("dgrad", dgr), ("mio_fwd", mf), ("mio_dgrad", md))
        t = {k: kbench.timeit(f, 20) * 1e3 for k, f in passes}
        fl = 2.0 * 9 * n * ho * wo * ci * co
        fwd()
        if ci == 3:  # the stem: the image needs no data gradient
            t["dgrad"] = t["mio_dgrad"] = 1e-9
            err = float((y - mf()).abs().max() / mf().abs().max())
        else:
            dgr()
            err = max(float((a - b).abs().max() / b.abs().max())
                      for a, b in ((y, mf()), (gx, md()[0])))
        tot["hip"] += uses * (t["fwd"] + t["dgrad"])
        tot["miopen"] += uses * (t["mio_fwd"] + t["mio_dgrad"])
        print(f"3x3s2 {ci}->{co} {h}x{w}: HIP fwd {t['fwd']:6.1f} dgrad {t['dgrad']:6.1f} us "
              f"({fl / t['fwd'] / 1e6:5.1f} / {fl / t['dgrad'] / 1e6:5.1f} TF/s) | MIOpen fwd "
              f"{t['mio_fwd']:6.1f} dgrad {t['mio_dgrad']:6.1f} us | rel diff {err:.1e}", flush=True)
    print(f"3x3s2 per cfg2 step (x uses): HIP {tot['hip']:.0f} us, MIOpen {tot['miopen']:.0f} us",
          flush=True)
    tot = {"hip": 0.0, "miopen": 0.0}
    for ci, co, h, w, uses in S1_SHAPES:
        x = torch.rand((n, ci, h, w), device="cuda") - 0.5
        wt = (torch.rand((co, ci, 3, 3), device="cuda") - 0.5) * 0.1
        gy = torch.rand((n, co, h, w), device="cuda") - 0.5
        y = torch.empty_like(gy)
        gx = torch.empty_like(x)
        st = _abi.stream_of(x)
        fwd = lambda: _abi.call("mde_conv3x3_wide_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, ci,
                                co, h, w, 0, st)
        dgr = lambda: _abi.call("mde_conv3x3_wide_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx),
                                n, ci, co, h, w, 0, st)
        mf = lambda: torch.nn.functional.conv2d(x, wt, None, 1, 1)
        md = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (1, 1), (1, 1),
                                                         False, (0, 0), 1, (True, False, False))
        u = torch.empty(_abi.query("mde_wino_weight_bytes", ci, co) // 4, device="cuda")
        yw = torch.empty_like(y)
        gxw = torch.empty_like(gx)

        def wf():  # Winograd forward incl. its weight transform
            _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), ci, co, 0, st)
            _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(yw), n, ci, co, h, w, 0, 0,
                      st)

        def wd():
            _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), ci, co, 1, st)
            _abi.call("mde_wino_conv", _abi.ptr(gy), _abi.ptr(u), _abi.ptr(gxw), n, co, ci, h, w, 1,
                      0, st)
        t = {k: kbench.timeit(f, 20) * 1e3 for k, f in
             (("fwd", fwd), ("dgrad", dgr), ("mio_fwd", mf), ("mio_dgrad", md), ("wino_fwd", wf),
              ("wino_dgrad", wd))}
        fl = 2.0 * 9 * n * h * w * ci * co
        fwd()
        dgr()
        wf()
        wd()
        ym, gxm = mf(), md()[0]
        err = max(float((a - b).abs().max() / b.abs().max()) for a, b in ((y, ym), (gx, gxm)))
        errw = max(float((a - b).abs().max() / b.abs().max()) for a, b in ((yw, ym), (gxw, gxm)))
        tot["hip"] += uses * (t["fwd"] + t["dgrad"])
        tot["miopen"] += uses * (t["mio_fwd"] + t["mio_dgrad"])
        tot["wino"] = tot.get("wino", 0.0) + uses * (t["wino_fwd"] + t["wino_dgrad"])
        print(f"3x3s1 {ci}->{co} {h}x{w}: band fwd {t['fwd']:6.1f} dgrad {t['dgrad']:6.1f} us "
              f"({fl / t['fwd'] / 1e6:5.1f} / {fl / t['dgrad'] / 1e6:5.1f} TF/s) | Winograd fwd "
              f"{t['wino_fwd']:6.1f} dgrad {t['wino_dgrad']:6.1f} us | MIOpen fwd "
              f"{t['mio_fwd']:6.1f} dgrad {t['mio_dgrad']:6.1f} us | rel diff {err:.1e} / {errw:.1e}",
              flush=True)
    print(f"3x3s1 per cfg2 step (x uses): band {tot['hip']:.0f} us, Winograd {tot['wino']:.0f} us, "
          f"MIOpen {tot['miopen']:.0f} us", flush=True)
    # the decoder's 16 -> 16 convs at 480 x 640: the direct MFMA kernel (with its
    # BN-statistics epilogue off) vs Winograd
    for ci, co, h, w in ((16, 16, 480, 640), (32, 32, 240, 320)):
        x = torch.rand((n, ci, h, w), device="cuda") - 0.5
        wt = (torch.rand((co, ci, 3, 3), device="cuda") - 0.5) * 0.1
        gy = torch.rand((n, co, h, w), device="cuda") - 0.5
        y, yw = torch.empty_like(gy), torch.empty_like(gy)
        gx, gxw = torch.empty_like(x), torch.empty_like(x)
        u = torch.empty(_abi.query("mde_wino_weight_bytes", ci, co) // 4, device="cuda")
        st = _abi.stream_of(x)
        fl = 2.0 * 9 * n * h * w * ci * co

        def df():
            _abi.call("mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, ci, co, h, w, 0, st)

        def dd():
            _abi.call("mde_conv3x3_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, ci, co, h,
                      w, 0, st)

        def wf():
            _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), ci, co, 0, st)
            _abi.call("mde_wino_conv", _abi.ptr(x), _abi.ptr(u), _abi.ptr(yw), n, ci, co, h, w, 0, 0,
                      st)

        def wd():
            _abi.call("mde_wino_weight", _abi.ptr(wt), _abi.ptr(u), ci, co, 1, st)
            _abi.call("mde_wino_conv", _abi.ptr(gy), _abi.ptr(u), _abi.ptr(gxw), n, co, ci, h, w, 1,
                      0, st)
        mf = lambda: torch.nn.functional.conv2d(x, wt, None, 1, 1)
        have_direct = bool(_abi.query("mde_conv3x3_supported", ci, co, 0, 0))
        fns = (("wino_fwd", wf), ("wino_dgrad", wd), ("mio_fwd", mf))
        if have_direct:
            fns = fns + (("fwd", df), ("dgrad", dd))
        t = {k: kbench.timeit(f, 20) * 1e3 for k, f in fns}
        wf()
        wd()
        ym = mf()
        gxm = torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (1, 1), (1, 1), False,
                                                  (0, 0), 1, (True, False, False))[0]
        errw = max(float((a - b).abs().max() / b.abs().max()) for a, b in ((yw, ym), (gxw, gxm)))
        direct = (f"direct fwd {t['fwd']:6.1f} dgrad {t['dgrad']:6.1f} us | " if have_direct else "")
        print(f"3x3s1 {ci}->{co} {h}x{w}: {direct}Winograd fwd {t['wino_fwd']:6.1f} "
              f"({fl / t['wino_fwd'] / 1e6:5.1f} TF/s eff.) dgrad {t['wino_dgrad']:6.1f} us | MIOpen "
              f"fwd {t['mio_fwd']:6.1f} us | Winograd rel diff {errw:.1e}", flush=True)


if __name__ == "__main__":
    main()
