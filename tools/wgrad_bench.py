"""Weight gradient of DDRNet's wide 3x3 convs at cfg2 (bs 32): the NCHW HIP
wide-channel kernel (mde_conv3x3_wgrad, incl. its reduction) vs MIOpen's
(aten.convolution_backward, NCHW tensors: incl. its layout transposes)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from monocular_depth_estimation_amd import _abi
from monocular_depth_estimation_amd.nn import _ws


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


tag = os.environ.get("MDE_WIDE_WPB", "8") + ("" if os.environ.get("MDE_C32_WIDE", "1") != "0" else " c32 off")
SHAPES = [(32, 64, 64, 60, 80), (32, 128, 128, 30, 40), (32, 256, 256, 15, 20),
          (32, 128, 64, 60, 80), (32, 64, 64, 120, 160), (4, 64, 64, 30, 40),
          (32, 32, 32, 120, 160), (32, 32, 32, 240, 320)]
if "--newcrf" in sys.argv:  # cfg4's NewCRF proj_v / proj_x convs (bs 16, newcrf_layers.py:377-379)
    SHAPES = [(16, 64, 128, 120, 160), (16, 128, 256, 60, 80), (16, 256, 512, 30, 40),
              (16, 512, 1024, 15, 20), (16, 160, 1024, 15, 20)]
ONLY = None  # --only n,c,co,h,w: that shape alone (profiling runs), no stride-2 sections
if "--only" in sys.argv:
    ONLY = tuple(int(v) for v in sys.argv[sys.argv.index("--only") + 1].split(","))
    SHAPES = [ONLY]
for (n, c, co, h, w) in SHAPES:
    x = torch.rand((n, c, h, w), device="cuda") - 0.5
    gy = torch.rand((n, co, h, w), device="cuda") - 0.5
    wt = torch.rand((co, c, 3, 3), device="cuda")
    gw = torch.empty_like(wt)
    ws = _ws(_abi.query("mde_conv3x3_wgrad_workspace", n, c, co, h, w, 0), x)
    st = _abi.stream_of(x)
    hip = lambda: _abi.call("mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, c, co,
                            h, w, _abi.ptr(ws), 0, st)
    mio = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (1, 1), (1, 1), False,
                                                      (0, 0), 1, (False, True, False))
    th, tm = timeit(hip), timeit(mio)
    hip()
    ref = mio()[1]
    err = float((gw - ref).abs().max() / ref.abs().max())
    fl = 2.0 * 9 * c * co * n * h * w
    print(f"[wpb {tag}] wgrad {c}->{co} {n}x{h}x{w}: HIP {th:7.1f} us ({fl / th / 1e6:5.1f} TF/s)  "
          f"MIOpen {tm:7.1f} us ({fl / tm / 1e6:5.1f} TF/s)  rel diff {err:.1e}", flush=True)

# stride-2 stem convolutions (mde_conv3x3s2_wgrad) vs MIOpen (incl. its NHWC transposes)
for (n, c, co, h, w) in ([] if "--newcrf" in sys.argv or ONLY else [(32, 3, 32, 480, 640), (32, 32, 32, 240, 320)]):
    x = torch.rand((n, c, h, w), device="cuda") - 0.5
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    gy = torch.rand((n, co, ho, wo), device="cuda") - 0.5
    wt = torch.rand((co, c, 3, 3), device="cuda")
    gw = torch.empty_like(wt)
    ws = _ws(_abi.query("mde_conv3x3s2_wgrad_workspace", n, c, co, h, w, 0), x)
    st = _abi.stream_of(x)
    hip = lambda: _abi.call("mde_conv3x3s2_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, c,
                            co, h, w, _abi.ptr(ws), 0, st)
    mio = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (2, 2), (1, 1), (1, 1), False,
                                                      (0, 0), 1, (False, True, False))
    th, tm = timeit(hip), timeit(mio)
    hip()
    ref = mio()[1]
    err = float((gw - ref).abs().max() / ref.abs().max())
    fl = 2.0 * 9 * c * co * n * ho * wo
    gb = 4.0 * n * (c * h * w + co * ho * wo) / 1e9
    print(f"[s2] wgrad {c}->{co} {n}x{h}x{w}: HIP {th:7.1f} us ({fl / th / 1e6:5.1f} TF/s, "
          f"{gb / th * 1e6:6.0f} GB/s)  MIOpen {tm:7.1f} us  rel diff {err:.1e}", flush=True)

# stride-2 wide weight gradients (DDRNet's stride-2 BasicBlock convs, down3 / down4)
for (n, c, co, h, w) in ([] if ONLY else [(32, 32, 64, 120, 160), (32, 64, 128, 60, 80), (32, 128, 256, 30, 40)]):
    x = torch.rand((n, c, h, w), device="cuda") - 0.5
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    gy = torch.rand((n, co, ho, wo), device="cuda") - 0.5
    wt = torch.rand((co, c, 3, 3), device="cuda")
    gw = torch.empty_like(wt)
    ws = _ws(_abi.query("mde_conv3x3s2_wgrad_workspace", n, c, co, h, w, 0), x)
    st = _abi.stream_of(x)
    hip = lambda: _abi.call("mde_conv3x3s2_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, c,
                            co, h, w, _abi.ptr(ws), 0, st)
    mio = lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (2, 2), (1, 1), (1, 1), False,
                                                      (0, 0), 1, (False, True, False))
    th, tm = timeit(hip), timeit(mio)
    hip()
    ref = mio()[1]
    err = float((gw - ref).abs().max() / ref.abs().max())
    fl = 2.0 * 9 * c * co * n * ho * wo
    print(f"[s2 wide] wgrad {c}->{co} {n}x{h}x{w}: HIP {th:7.1f} us ({fl / th / 1e6:5.1f} TF/s)  "
          f"MIOpen {tm:7.1f} us  rel diff {err:.1e}", flush=True)
