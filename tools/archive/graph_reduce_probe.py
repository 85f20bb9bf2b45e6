"""Does an ATen column reduction replayed from a HIP graph read stale / unwritten memory?

Inside the captured region a NaN-filled scratch tensor is freed right before
`x.sum(0)`, so the reduction's staging buffer (global reduce over many rows)
is likely carved from the same pool memory.  Each replay is compared with the
eager result.  Debug aid for the bf16 Linear-bias gradient issue.
"""
import sys

import torch

dev = torch.device("cuda")
torch.manual_seed(0)
cases = [(4800, 2048), (19200, 2048), (76800, 1024), (76800, 512), (4800, 4096)]
bad_any = False
for dtype in (torch.bfloat16, torch.float32):
    for rows, cols in cases:
        x = torch.randn(rows, cols, device=dev).to(dtype)
        ref = x.float().sum(0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up
                t = torch.full((rows * cols // 2,), float("nan"), device=dev)
                del t
                y = x.sum(0)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            t = torch.full((rows * cols // 2,), float("nan"), device=dev)
            del t
            y = x.sum(0)
            t2 = torch.full((rows * cols // 2,), float("nan"), device=dev)
            del t2
        res = []
        for r in range(6):
            g.replay()
            torch.cuda.synchronize()
            err = (y.float() - ref).abs().max().item()
            nf = (~torch.isfinite(y)).sum().item()
            res.append((round(err, 4), nf))
        tol = 0.05 * ref.abs().max().item() if dtype == torch.bfloat16 else 1e-2
        bad = any(nf or err > tol for err, nf in res)
        bad_any |= bad
        print(f"{str(dtype):15s} {rows}x{cols}: replays (max err, non-finite) {res}"
              f"{'  <-- BAD' if bad else ''}", flush=True)
        del g

# the Linear-bias gradient itself, captured fwd+bwd, in several variants
def bias_case(rows, cin, cout, variant):
    lin = torch.nn.Linear(cin, cout).to(dev)
    x = torch.randn(1, rows, cin, device=dev)
    go = torch.randn(1, rows, cout, device=dev)
    amp = variant in ("amp", "amp_addb", "amp_rocblas")
    if variant == "amp_rocblas":
        torch.backends.cuda.preferred_blas_library("cublas")

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            if variant == "amp_addb":
                y = torch.nn.functional.linear(x, lin.weight) + lin.bias
            else:
                y = lin(x)
        y.backward(go.to(y.dtype))

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            lin.zero_grad(set_to_none=True)
            run()
    torch.cuda.current_stream().wait_stream(s)
    ref = lin.bias.grad.clone()
    lin.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    res = []
    for r in range(4):
        g.replay()
        torch.cuda.synchronize()
        gb = lin.bias.grad
        ratio = float((gb * ref).sum() / (ref * ref).sum())
        res.append((round((gb - ref).abs().max().item(), 3), round(ratio, 3)))
    torch.backends.cuda.preferred_blas_library("default")
    bad = any(e > 0.05 * ref.abs().max().item() for e, _ in res)
    print(f"linear bias grad {variant:12s} {rows}x{cin}->{cout}: (max err, <g,ref>/<ref,ref>) {res}"
          f"{'  <-- BAD' if bad else ''}", flush=True)
    return bad


for variant in ("fp32", "amp", "amp_addb", "amp_rocblas"):
    for rows, cin, cout in [(4800, 1024, 4096), (76800, 256, 1024)]:
        bad_any |= bias_case(rows, cin, cout, variant)
sys.exit(1 if bad_any else 0)
