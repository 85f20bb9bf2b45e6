"""A/B: pointwise (BN-ReLU fused) backward + BN backward, unfused reduce vs the
BNS epilogue (mde_pointwise_bwd_bn + mde_batchnorm_bwd_apply), cfg2 shapes."""
import json
import sys

import torch

sys.path.insert(0, ".")
from monocular_depth_estimation_amd import _abi  # noqa: E402

SHAPES = [(16, 8, 32, 480, 640), (32, 16, 32, 240, 320), (64, 32, 32, 120, 160)]


def main():
    f = dict(device="cuda", dtype=torch.float32)
    res = {}
    for cin, cout, n, h, w in SHAPES:
        y1 = torch.rand((n, cin, h, w), **f) * 2 - 0.7
        gy2 = torch.rand((n, cout, h, w), **f) - 0.5
        w2 = torch.rand((cout, cin), **f) - 0.5
        gamma, beta = torch.rand(cin, **f) + 0.5, torch.rand(cin, **f) - 0.5
        mean = y1.mean(dim=(0, 2, 3))
        invstd = 1.0 / torch.sqrt(y1.var(dim=(0, 2, 3), unbiased=False) + 1e-5)
        scale = gamma * invstd
        shift = beta - mean * scale
        st = _abi.stream_of(y1)
        ws = torch.empty(_abi.query("mde_pointwise_workspace", n, cin, cout, h, w) // 4 + 1, **f)
        ws2 = torch.empty(_abi.query("mde_batchnorm_workspace", n, cin, h, w) // 4 + 1, **f)
        gz, gw2, gy1 = torch.empty_like(y1), torch.empty_like(w2), torch.empty_like(y1)
        gg, gb, sums = torch.empty(cin, **f), torch.empty(cin, **f), torch.empty((cin, 2), **f)

        def unfused():
            _abi.call("mde_pointwise_bwd", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(w2), _abi.ptr(gz), _abi.ptr(gw2), n, cin, cout, h,
                      w, _abi.ptr(ws), 0, st)

        def unfused_bn():
            _abi.call("mde_batchnorm_bwd", _abi.ptr(gz), _abi.ptr(y1), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(gy1), None,
                      _abi.ptr(gg), _abi.ptr(gb), None, n, cin, h, w, 1, _abi.ptr(ws2), 0, st)

        def fused():
            _abi.call("mde_pointwise_bwd_bn", _abi.ptr(gy2), _abi.ptr(y1), _abi.ptr(scale),
                      _abi.ptr(shift), _abi.ptr(mean), _abi.ptr(w2), _abi.ptr(gz), _abi.ptr(gw2),
                      _abi.ptr(sums), n, cin, cout, h, w, _abi.ptr(ws), 0, st)

        def fused_bn():
            _abi.call("mde_batchnorm_bwd_apply", _abi.ptr(gz), _abi.ptr(y1), None, _abi.ptr(gamma),
                      _abi.ptr(beta), _abi.ptr(mean), _abi.ptr(invstd), 1, _abi.ptr(sums),
                      _abi.ptr(gy1), None, _abi.ptr(gg), _abi.ptr(gb), None, n, cin, h, w, 1, 0, st)

        def t(fn, reps=20):
            for _ in range(3):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) * 1e3 / reps

        r = {"pw_bwd": t(unfused), "bn_bwd": t(unfused_bn)}
        if cin <= 32:
            r.update(pw_bwd_bn=t(fused), bn_apply=t(fused_bn))
            r["fused_total"] = r["pw_bwd_bn"] + r["bn_apply"]
        r["unfused_total"] = r["pw_bwd"] + r["bn_bwd"]
        key = f"{cin}->{cout} {n}x{h}x{w}"
        res[key] = {k: round(v, 1) for k, v in r.items()}
        print(key, res[key], flush=True)
    json.dump(res, open("gpurun_out/pw_bn_bench.json", "w"), indent=1)


if __name__ == "__main__":
    main()
