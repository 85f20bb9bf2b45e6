"""Per-op micro-benchmark of the HIP kernels at GuideDepth cfg2 shapes (640x480, bs=32).

    python tools/kbench.py [--reps 20]

Times each op's forward and backward from HIP-graph replays (10 calls per graph) over `reps`
back-to-back calls (after 3 warm-ups) and prints algorithmic GB/s (SURVEY
§8(d) byte formulas) against the 8 TB/s HBM peak.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_STREAM = None  # every op, its forward for a backward timing, and the captures run here


def timeit(fn, reps):
    """ms per call of fn, from replays of a HIP graph holding 10 calls (device
    time without the host's launch overhead).  The graph is captured on the
    stream main() runs everything on, which is also the stream the autograd
    backward of a forward made there launches on."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    inner = 10
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=_STREAM):
        for _ in range(inner):
            fn()
    outer = max(1, reps // inner)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(outer):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (outer * inner)


def main():
    global _STREAM
    _STREAM = torch.cuda.Stream()
    with torch.cuda.stream(_STREAM):
        _main()


def _main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--only", default="", help="comma list of groups: resize,se,skip,pw,bn,loss,attn,dw,ln")
    a = ap.parse_args()
    groups = set(a.only.split(",")) if a.only else None

    def want(g):
        return groups is None or g in groups
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd import functional as F
    from monocular_depth_estimation_amd.nn import BatchNorm2d
    dev = "cuda"
    rows = []

    def report(name, ms, nbytes):
        gbs = nbytes / (ms * 1e-3) / 1e9
        rows.append({"op": name, "ms": round(ms, 4), "GBps": round(gbs, 1), "frac": round(gbs / 8000, 3)})
        print(f"{name:44s} {ms * 1e3:9.1f} us {gbs:8.1f} GB/s  {gbs / 8000:6.1%}", flush=True)

    n = 32
    # bilinear x2 (decoder) and DDRNet resizes
    for c, h, w in ((64, 60, 80), (32, 120, 160), (16, 240, 320)) if want("resize") else ():
        x = torch.rand(n, c, h, w, device=dev)
        y = F.bilinear_resize(x, scale_factor=2)
        gy = torch.rand_like(y)
        nb = 4.0 * n * c * (h * w + 4 * h * w)
        report(f"bilinear_fwd x2 {c}x{h}x{w}", timeit(lambda: F.bilinear_resize(x, scale_factor=2), a.reps), nb)
        ho, wo = 2 * h, 2 * w
        report(f"bilinear_bwd x2 {c}x{h}x{w}", timeit(lambda: _abi.call(
            "mde_bilinear_bwd", gy.data_ptr(), x.data_ptr(), n, c, h, w, ho, wo, 0.5, 0.5, 0, 0,
            _abi.stream_of(x)), a.reps), nb)
    # the same x2 upsample on bf16 storage (cfg3 autocast): half the bytes
    for c, h, w in ((64, 60, 80), (32, 120, 160), (16, 240, 320)) if want("resize") else ():
        x = torch.rand(n, c, h, w, device=dev).to(torch.bfloat16)
        gy = torch.rand(n, c, 2 * h, 2 * w, device=dev).to(torch.bfloat16)
        gx = torch.empty_like(x)
        nb = 2.0 * n * c * (h * w + 4 * h * w)
        report(f"bilinear_fwd x2 bf16 {c}x{h}x{w}",
               timeit(lambda: F.bilinear_resize(x, scale_factor=2), a.reps), nb)
        report(f"bilinear_bwd x2 bf16 {c}x{h}x{w}", timeit(lambda: _abi.call(
            "mde_bilinear_bwd", gy.data_ptr(), gx.data_ptr(), n, c, h, w, 2 * h, 2 * w, 0.5, 0.5, 0,
            1, _abi.stream_of(x)), a.reps), nb)
    for c, hi, wi in ((64, 15, 20), (128, 8, 10)) if want("resize") else ():
        x = torch.rand(n, c, hi, wi, device=dev)
        nb = 4.0 * n * c * (hi * wi + 60 * 80)
        report(f"bilinear_fwd {c}x{hi}x{wi}->60x80", timeit(lambda: F.bilinear_resize(x, size=(60, 80)), a.reps), nb)
        gy = torch.rand(n, c, 60, 80, device=dev)
        report(f"bilinear_bwd {c}x{hi}x{wi}->60x80", timeit(lambda: _abi.call(
            "mde_bilinear_bwd", gy.data_ptr(), x.data_ptr(), n, c, hi, wi, 60, 80, hi / 60, wi / 80,
            0, 0, _abi.stream_of(x)), a.reps), nb)
    if want("resize"):  # NewCRF head: sigmoid map x4 (cfg4, bs 16)
        x = torch.rand(16, 1, 120, 160, device=dev)
        nb = 4.0 * 16 * (120 * 160 + 480 * 640)
        report("bilinear_fwd x4 1x120x160 (bs16)", timeit(lambda: F.bilinear_resize(x, scale_factor=4),
                                                         a.reps), nb)
        gy = torch.rand(16, 1, 480, 640, device=dev)
        report("bilinear_bwd x4 1x120x160 (bs16)", timeit(lambda: _abi.call(
            "mde_bilinear_bwd", gy.data_ptr(), x.data_ptr(), 16, 1, 120, 160, 480, 640, 0.25, 0.25,
            0, 0, _abi.stream_of(x)), a.reps), nb)
    if want("resize"):
        img = torch.rand(n, 3, 480, 640, device=dev)
        for sf in (0.5, 0.25):
            ho, wo = int(480 * sf), int(640 * sf)
            report(f"nearest_fwd x{sf} 3x480x640", timeit(lambda: F.nearest_resize(img, scale_factor=sf),
                                                          a.reps), 8.0 * n * 3 * ho * wo)
        report("nearest_pyramid x0.5+x0.25 3x480x640", timeit(lambda: F.nearest_pyramid(img), a.reps),
               8.0 * n * 3 * (240 * 320 + 120 * 160))
    # decoder pointwise 1x1 convs (E -> E/2, BN + ReLU on the operand load,
    # the next BN's statistics from the epilogue), forward
    for c, co, h, w in ((64, 64, 120, 160), (64, 32, 120, 160), (32, 16, 240, 320), (16, 8, 480, 640)) \
            if want("pw") else ():
        x = torch.rand(n, c, h, w, device=dev)
        wt = torch.rand(co, c, device=dev) - 0.5
        sc, sh = torch.rand(c, device=dev), torch.rand(c, device=dev) - 0.5
        y = torch.empty(n, co, h, w, device=dev)
        nb = _abi.query("mde_pointwise_stats_blocks", n, c, co, h, w)
        st = torch.empty(co * nb * 4, device=dev)
        report(f"pointwise fwd bnr+stats {c}->{co} {h}x{w}", timeit(lambda: _abi.call(
            "mde_pointwise_fwd_stats", x.data_ptr(), sc.data_ptr(), sh.data_ptr(), wt.data_ptr(),
            y.data_ptr(), st.data_ptr(), n, c, co, h, w, 0, _abi.stream_of(x)), a.reps),
            4.0 * n * h * w * (c + co))
    # SE + cat and skip fusion at the three decoder resolutions
    for c, h, w, cout in ((64, 120, 160, 32), (32, 240, 320, 16), (16, 480, 640, 1)) \
            if (want("se") or want("skip")) else ():
        half = c // 2
        xa = torch.rand(n, half, h, w, device=dev)
        xb = torch.rand(n, half, h, w, device=dev)
        w1 = torch.rand(c, c, device=dev) * 0.1
        w2 = torch.rand(c, c, device=dev) * 0.1
        big = 4.0 * n * c * h * w
        report(f"se_cat fwd {c}x{h}x{w}", timeit(lambda: F.se_cat(xa, xb, w1, w2), a.reps), 3 * big)
        xa.requires_grad_(True)
        xb.requires_grad_(True)
        out = F.se_cat(xa, xb, w1, w2)
        g = torch.rand_like(out)
        report(f"se_cat bwd {c}x{h}x{w}",
               timeit(lambda: torch.autograd.grad(out, (xa, xb), g, retain_graph=True), a.reps), 4 * big)
        r = torch.rand(n, c, h, w, device=dev)
        d = torch.rand(n, c, h, w, device=dev)
        wt = torch.rand(cout, c, 1, 1, device=dev)
        b = torch.rand(cout, device=dev)
        pix = n * h * w * 4.0
        report(f"skip_reduce fwd {c}->{cout} {h}x{w}", timeit(lambda: F.skip_reduce(r, d, wt, b), a.reps),
               pix * (2 * c + cout))
        r.requires_grad_(True)
        wt.requires_grad_(True)
        o = F.skip_reduce(r, d, wt, b)
        go = torch.rand_like(o)
        report(f"skip_reduce bwd {c}->{cout} {h}x{w}",
               timeit(lambda: torch.autograd.grad(o, (r, wt), go, retain_graph=True), a.reps),
               pix * (3 * c + cout))
    # BatchNorm(+ReLU) at representative shapes
    for c, h, w in ((16, 480, 640), (32, 240, 320), (16, 240, 320), (64, 120, 160), (32, 120, 160),
                    (64, 60, 80), (256, 15, 20)) if want("bn") else ():
        x = torch.rand(n, c, h, w, device=dev, requires_grad=True)
        bn = BatchNorm2d(c, act="relu").to(dev).train()
        big = 4.0 * n * c * h * w
        report(f"bn+relu fwd {c}x{h}x{w}", timeit(lambda: bn(x), a.reps), 3 * big)
        y = bn(x)
        gy = torch.rand_like(y)
        report(f"bn+relu bwd {c}x{h}x{w}",
               timeit(lambda: torch.autograd.grad(y, (x,), gy, retain_graph=True), a.reps), 5 * big)
        ref = torch.nn.BatchNorm2d(c).to(dev).train()
        report(f"  (MIOpen BN fwd {c}x{h}x{w})", timeit(lambda: ref(x), a.reps), 3 * big)
    # loss
    if want("loss"):
        p = torch.rand(n, 1, 480, 640, device=dev, requires_grad=True)
        t = torch.rand(n, 1, 480, 640, device=dev) * 10
        mm = F.minmax(t)
        report("ssim3_l1 fwd+grad 480x640", timeit(lambda: F.ssim3_l1(p, t, 1.0, 0.1, target_minmax=mm),
                                                   a.reps), 3 * 4.0 * n * 480 * 640)
        report("minmax 480x640", timeit(lambda: F.minmax(t), a.reps), 4.0 * n * 480 * 640)
        # GuideDepth Depth_Loss (losses.py:15-127), Alhashim mode (0.1, 1, 1), fwd + bwd:
        # algorithmic bytes = pred + gt read by the forward, pred + gt read and
        # grad written by the backward (the per-pixel coefficient map of the 11x11
        # SSIM backward is an intermediate, 3 planes written + read, counted too)
        dl_bytes = 4.0 * n * 480 * 640 * (2 + 3 + 6)
        report("depth_loss fwd+bwd (0.1,1,1) 480x640",
               timeit(lambda: torch.autograd.grad(F.depth_loss(p, t, 0.1, 1.0, 1.0, 10.0)[0], (p,)),
                      a.reps), dl_bytes)
        report("depth_loss fwd+bwd masked L1 (1,0,0) 480x640",
               timeit(lambda: torch.autograd.grad(F.depth_loss(p, t, 1.0, 0.0, 0.0, 10.0)[0], (p,)),
                      a.reps), 4.0 * n * 480 * 640 * 5)
        from monocular_depth_estimation_amd.data import nyu_augment
        img_u8 = torch.randint(0, 256, (n, 480, 640, 3), dtype=torch.uint8, device=dev)
        dep_u8 = torch.randint(0, 256, (n, 480, 640), dtype=torch.uint8, device=dev)
        flg = torch.tensor([(i % 2, i % 7 - 1) for i in range(n)], dtype=torch.int32, device=dev)
        report("nyu_augment 32x480x640 (uint8 -> fp32)",
               timeit(lambda: nyu_augment(img_u8, dep_u8, flg), a.reps), 20.0 * n * 480 * 640)
        crop = F.eigen_crop(480, 640)
        report("eval_sums (test.py batch) 480x640",
               timeit(lambda: F.eval_sums(p.detach(), t, 1e-3, 80.0, True, crop), a.reps),
               8.0 * n * 480 * 640)
    # --- cfg4 (PTModel, bs 16) ops
    n4 = 16
    if want("attn"):
        from monocular_depth_estimation_amd.newcrf_layers import window_attention
        for c, heads, h, w in ((128, 4, 120, 160), (256, 8, 60, 80), (512, 16, 30, 40), (1024, 32, 15, 20)):
            qk = torch.randn(n4, h * w, 2 * c, device=dev, requires_grad=True)
            qkb = torch.randn(2 * c, device=dev, requires_grad=True)
            v = torch.randn(n4, h, w, c, device=dev, requires_grad=True)
            tab = torch.randn(169, heads, device=dev, requires_grad=True)
            tok = 4.0 * n4 * h * w * c
            for shift in (0, 3):
                report(f"window_attn fwd C{c} {h}x{w} s{shift}",
                       timeit(lambda: window_attention(qk, qkb, v, tab, h, w, heads, 7, shift), a.reps),
                       4 * tok)
                o = window_attention(qk, qkb, v, tab, h, w, heads, 7, shift)
                go = torch.randn_like(o)
                report(f"window_attn bwd C{c} {h}x{w} s{shift}",
                       timeit(lambda: torch.autograd.grad(o, (qk, v, tab, qkb), go, retain_graph=True),
                              a.reps), 7 * tok)
    if want("dw"):
        from monocular_depth_estimation_amd.nn import depthwise_conv2d
        # every depthwise stage of MobileNetV3-Large at 480x640 (features[1..15]; x2 = repeated)
        for c, h, w, k, st in ((16, 240, 320, 3, 1), (64, 240, 320, 3, 2), (72, 120, 160, 3, 1),
                               (72, 120, 160, 5, 2), (120, 60, 80, 5, 1), (240, 60, 80, 3, 2),
                               (200, 30, 40, 3, 1), (184, 30, 40, 3, 1), (480, 30, 40, 3, 1),
                               (672, 30, 40, 3, 1), (672, 30, 40, 5, 2), (960, 15, 20, 5, 1)):
            conv = torch.nn.Conv2d(c, c, k, st, k // 2, groups=c, bias=False).to(dev)
            x = torch.randn(n4, c, h, w, device=dev, requires_grad=True)
            y = depthwise_conv2d(x, conv)
            gy = torch.randn_like(y)
            nb = 4.0 * (x.numel() + y.numel())
            report(f"dwconv fwd {c}x{h}x{w} k{k}s{st}", timeit(lambda: depthwise_conv2d(x, conv), a.reps), nb)
            report(f"dwconv bwd {c}x{h}x{w} k{k}s{st}",
                   timeit(lambda: torch.autograd.grad(y, (x, conv.weight), gy, retain_graph=True),
                          a.reps), 4.0 * (2 * x.numel() + y.numel()))  # gy + x read, gx written
    if want("ln"):
        from monocular_depth_estimation_amd.newcrf_layers import LayerNorm, nchw_to_tokens
        for c, h, w in ((128, 120, 160), (256, 60, 80), (512, 30, 40), (1024, 15, 20)):
            ln = LayerNorm(c).to(dev)
            x = torch.randn(n4, h * w, c, device=dev, requires_grad=True)
            y = ln(x)
            gy = torch.randn_like(y)
            nb = 4.0 * x.numel()
            report(f"layernorm fwd {c} {h}x{w}", timeit(lambda: ln(x), a.reps), 2 * nb)
            report(f"layernorm bwd {c} {h}x{w}",
                   timeit(lambda: torch.autograd.grad(y, (x, ln.weight), gy, retain_graph=True), a.reps),
                   3 * nb)
            xn = torch.randn(n4, c, h, w, device=dev)
            report(f"transpose nchw->tokens {c} {h}x{w}", timeit(lambda: nchw_to_tokens(xn), a.reps), 2 * nb)
    if want("conv"):
        # HIP MFMA 3x3 conv vs MIOpen, per pass, at the cfg2 shapes (bs 32);
        # `frac` here is of the 157.3 TFLOP/s fp32 MFMA peak, GBps is algorithmic bytes.
        def report_tf(name, ms, flop, nbytes):
            tf = flop / (ms * 1e-3) / 1e12
            rows.append({"op": name, "ms": round(ms, 4), "TFLOPs": round(tf, 1),
                         "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "frac": round(tf / 157.3, 3)})
            print(f"{name:44s} {ms * 1e3:9.1f} us {tf:8.1f} TF/s  {tf / 157.3:6.1%}", flush=True)
        tconv = torch.nn.functional.conv2d
        for cin, cout, h, w in ((3, 16, 480, 640), (16, 16, 480, 640), (3, 32, 240, 320),
                                (32, 32, 240, 320), (3, 64, 120, 160), (64, 64, 60, 80),
                                (64, 64, 120, 160)):
            x = torch.rand(n, cin, h, w, device=dev) - 0.5
            wt = torch.rand(cout, cin, 3, 3, device=dev) - 0.5
            gy = torch.rand(n, cout, h, w, device=dev) - 0.5
            y = torch.empty_like(gy)
            gx = torch.empty_like(x)
            gw = torch.empty_like(wt)
            ws = torch.empty(_abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w, 0) // 4 + 1,
                             device=dev)
            st = _abi.stream_of(x)
            flop = 2.0 * n * h * w * cout * cin * 9
            nb = 4.0 * n * h * w * (cin + cout)
            tag = f"{cin}->{cout} {h}x{w}"
            if _abi.query("mde_conv3x3_supported", cin, cout, 0, 0):
                report_tf(f"conv3x3 fwd HIP {tag}", timeit(lambda: _abi.call(
                    "mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, cin, cout, h, w, 0,
                    st), a.reps), flop, nb)
            report_tf(f"conv3x3 fwd MIOpen {tag}", timeit(lambda: tconv(x, wt, None, 1, 1), a.reps), flop, nb)
            if _abi.query("mde_conv3x3_supported", cin, cout, 1, 0):
                report_tf(f"conv3x3 dgrad HIP {tag}", timeit(lambda: _abi.call(
                    "mde_conv3x3_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, cin, cout, h, w,
                    0, st), a.reps), flop, nb)
                report_tf(f"conv3x3 dgrad MIOpen {tag}", timeit(
                    lambda: torch.nn.grad.conv2d_input(x.shape, wt, gy, padding=1), a.reps), flop, nb)
            if _abi.query("mde_conv3x3_supported", cin, cout, 2, 0):
                report_tf(f"conv3x3 wgrad HIP {tag}", timeit(lambda: _abi.call(
                    "mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin, cout, h,
                    w, _abi.ptr(ws), 0, st), a.reps), flop, nb)
            report_tf(f"conv3x3 wgrad MIOpen {tag}", timeit(
                lambda: torch.nn.grad.conv2d_weight(x, wt.shape, gy, padding=1), a.reps), flop, nb)
    if want("convbf"):
        # bf16 MFMA 3x3 convs (cfg3 autocast shapes, bs 32) vs MIOpen bf16; frac
        # of the 2.5 PF bf16 peak, GBps algorithmic (2-byte activations)
        def report_bf(name, ms, flop, nbytes):
            tf = flop / (ms * 1e-3) / 1e12
            gbs = nbytes / (ms * 1e-3) / 1e9
            rows.append({"op": name, "ms": round(ms, 4), "TFLOPs": round(tf, 1), "GBps": round(gbs, 1),
                         "frac": round(tf / 2516.6, 3), "hbm_frac": round(gbs / 8000, 3)})
            print(f"{name:44s} {ms * 1e3:9.1f} us {tf:8.1f} TF/s {gbs:7.0f} GB/s ({gbs / 8000:5.1%})",
                  flush=True)
        bf = torch.bfloat16
        tconv = torch.nn.functional.conv2d
        for cin, cout, h, w in ((16, 16, 480, 640), (32, 32, 240, 320), (32, 32, 120, 160)):
            x = (torch.rand(n, cin, h, w, device=dev) - 0.5).to(bf)
            wt = torch.rand(cout, cin, 3, 3, device=dev) - 0.5
            gy = (torch.rand(n, cout, h, w, device=dev) - 0.5).to(bf)
            y = torch.empty_like(gy)
            gx = torch.empty_like(x)
            gw = torch.empty_like(wt)
            ws = torch.empty(_abi.query("mde_conv3x3_wgrad_workspace", n, cin, cout, h, w, 1) // 4 + 1,
                             device=dev)
            st = _abi.stream_of(x)
            flop = 2.0 * n * h * w * cout * cin * 9
            nb = 2.0 * n * h * w * (cin + cout)
            tag = f"{cin}->{cout} {h}x{w}"
            report_bf(f"conv3x3 bf16 fwd HIP {tag}", timeit(lambda: _abi.call(
                "mde_conv3x3_fwd", _abi.ptr(x), _abi.ptr(wt), _abi.ptr(y), n, cin, cout, h, w, 1,
                st), a.reps), flop, nb)
            report_bf(f"conv3x3 bf16 dgrad HIP {tag}", timeit(lambda: _abi.call(
                "mde_conv3x3_bwd_data", _abi.ptr(gy), _abi.ptr(wt), _abi.ptr(gx), n, cin, cout, h, w,
                1, st), a.reps), flop, nb)
            report_bf(f"conv3x3 bf16 wgrad HIP {tag}", timeit(lambda: _abi.call(
                "mde_conv3x3_wgrad", _abi.ptr(gy), _abi.ptr(x), _abi.ptr(gw), n, cin, cout, h,
                w, _abi.ptr(ws), 1, st), a.reps), flop, nb)
            wb = wt.to(bf)
            report_bf(f"conv3x3 bf16 fwd MIOpen {tag}", timeit(lambda: tconv(x, wb, None, 1, 1), a.reps),
                      flop, nb)
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
