"""Per-kernel HIP-event timing inside a captured graph (debug aid for csrc/timing.hip)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from monocular_depth_estimation_amd import _abi  # noqa: E402
from monocular_depth_estimation_amd.functional import bilinear_resize, minmax  # noqa: E402

x = torch.rand(32, 16, 240, 320, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y = bilinear_resize(x, scale_factor=2)
    m = minmax(y)
torch.cuda.synchronize()
_abi.timing_reset()
_abi.timing_enable(True)
try:
    def body():
        yy = bilinear_resize(x, scale_factor=2)
        return minmax(yy)
    g, out, _ = _abi.capture_graph(body, s)
finally:
    _abi.timing_enable(False)
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    _abi.call("mde_timing_collect")
    print("after replay", r, {k: (round(v[0], 4), v[1]) for k, v in _abi.timing_collect(False).items()})
print("minmax", out.tolist(), float(x.min()), float(x.max()))
