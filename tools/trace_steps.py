"""Per-step kernel breakdown from a rocprofv3 kernel-trace CSV.

Steps are delimited by the `minmax_partial_kernel` launches (one per train
step, at the loss); the last K intervals are the timed steady state, which
excludes MIOpen's first-call solver search.  Usage:

    python tools/trace_steps.py gpurun_out/prof/trace/r01_kernel_trace.csv [--steps 4] [--top 40]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re

MARK = "minmax_partial_kernel"

OURS = re.compile(r"^(bilinear|nearest|se_partial|se_fc|se_scale|se_bfc|se_wgrad|se_apply|skip_|minmax|"
                  r"depthnorm|ssim3|loss_final|dloss|bn_|sebn_|wattn|dw_|ln_|conv3x3|wgrad_reduce|transpose_kernel|"
                  r"colsum|gelu_|nyu_|eval_|wino_|c3s2_|c3s1_|c1_|cm_kernel|convbf_|graph_fill|pwbf_|pw_bwd|stem_|c3in3)")


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    m = re.match(r"(?:mde::)?(?:\(anonymous namespace\)::)?(\w+)", name)
    base = m.group(1) if m else name[:60]
    if base.startswith("Cijk_"):
        return "rocBLAS/Tensile " + base[:48]
    if base == "at":
        m2 = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)<.*?(?:at::native::(?:\(anonymous namespace\)::)?(\w+))?", name)
        return "aten " + (m2.group(1) + ("/" + m2.group(2) if m2.group(2) else "") if m2 else name[:70])
    if base.startswith("_ZN2ck") or "ck::" in name:
        return "CK " + re.sub(r"^.*?(kernel_\w+).*$", r"\1", name)[:60]
    return base[:80]


def analyse(path: str, steps: int):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if MARK in r["Kernel_Name"]]
    if len(marks) < steps + 1:
        raise SystemExit(f"only {len(marks)} step markers")
    lo, hi = marks[-steps - 1], marks[-1]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo <= s < hi:
            k = short(r["Kernel_Name"])
            agg[k][0] += (e - s) / 1e6
            agg[k][1] += 1
    wall = (hi - lo) / 1e6 / steps
    busy = sum(v[0] for v in agg.values()) / steps
    ours = sum(v[0] for k, v in agg.items() if OURS.search(k)) / steps
    return wall, busy, ours, sorted(((v[0] / steps, v[1] / steps, k) for k, v in agg.items()), reverse=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    wall, busy, ours, table = analyse(a.csv, a.steps)
    print(f"per step: wall {wall:.2f} ms, kernel-busy {busy:.2f} ms, hand-written HIP {ours:.2f} ms")
    for ms, n, k in table[:a.top]:
        print(f"{ms:9.3f} ms/step {n:7.1f} calls  {k}")
    if a.json:
        json.dump({"wall_ms": wall, "busy_ms": busy, "hip_ms": ours,
                   "kernels": [{"name": k, "ms_per_step": ms, "calls_per_step": n} for ms, n, k in table]},
                  open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
