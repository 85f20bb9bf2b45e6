"""Is a hipMemsetAsync captured into a HIP graph re-executed correctly on every replay?

The captured sequence is memset(buf, 0) -> buf += 1 (a kernel); after each
replay buf must be all ones.  Run once as captured ("raw") and once after
mde_graph_replace_memsets ("repaired").  Debug aid / regression check for
csrc/graph.hip.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monocular_depth_estimation_amd import _abi  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int
dev = torch.device("cuda")
ok = True
for repaired in (False, True):
    for n in (4, 64, 4096, 1 << 20):
        buf = torch.zeros(n, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream()

        def body():
            hip.hipMemsetAsync(buf.data_ptr(), 0, n * 4, s.cuda_stream)
            buf.add_(1)

        if repaired:
            g, _, nrep = _abi.capture_graph(body, s)
        else:
            g, nrep = torch.cuda.CUDAGraph(), 0
            with torch.cuda.graph(g, stream=s):
                body()
        vals = []
        for r in range(4):
            g.replay()
            torch.cuda.synchronize()
            vals.append((int(buf.min()), int(buf.max())))
        good = all(v == (1, 1) for v in vals)
        if repaired:
            ok &= good and nrep == 1
        print(f"{'repaired' if repaired else 'raw':8s} memset {n * 4} B ({nrep} replaced): "
              f"after replays (min, max) {vals}{'' if good else '  <-- wrong'}", flush=True)
sys.exit(0 if ok else 1)
