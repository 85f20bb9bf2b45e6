"""HBM bytes per launch of the hand-written kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv [--last-steps 2] [-o profiles/r01_pmc_traffic.json]

FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit
one TCC pass).  Per MI355X_MICROARCH.md §HBM: both are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The guide states the x2 for 16-byte lanes only; tools/calib/pmc_calib (1 GiB
coalesced streams at 4-, 8- and 16-byte lanes, profiles/r03_pmc_calib.json)
measured FETCH factor 2.000 and WRITE factor 1.000 at EVERY width, so the
correction holds for this repo's narrow-lane kernels (ssim3_l1, the depth
loss, the BN table kernels) too: their ratios are real re-fetch.
Only the launches of the last K train steps are used (steady state: the K
steps between two minmax_partial_kernel launches -- the loss, mid-step).  Keys are the
timing-registry names bench.py reports (mde_kernel_name).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re

# demangled kernel symbol -> timing-registry name (csrc/timing.hip)
NAMES = [
    (r"bilinear_fwd\w*_kernel", "bilinear_fwd"),
    (r"bilinear_bwd\w*_kernel", "bilinear_bwd"),
    (r"nearest_(fwd|pyramid)_kernel", "nearest_fwd"),
    (r"nearest_bwd_kernel", "nearest_bwd"),
    # se_partial_kernel<mode, T>: 0 squeeze, 1 backward dot, 2 squeeze over BN + ReLU
    (r"se_partial_kernel<[02],", "se_squeeze"),
    (r"se_partial_kernel<1,", "se_bwd_dot"),
    (r"se_fc[12]_kernel", "se_fc"),
    (r"se_scale_kernel", "se_scale"),
    (r"se_(bfc[123]w?|bfc_all|wgrad)_kernel|sebn_bwd_combine_kernel", "se_bwd_fc"),
    (r"se_apply_kernel|sebn_bwd_apply_kernel", "se_bwd_apply"),
    # the SE-over-BN backward's reduction pass runs under the SE dot id (se.hip)
    (r"sebn_bwd_reduce_kernel", "se_bwd_dot"),
    (r"skip_fwd_mfma_kernel<\d+, \d+, true", "skip_reduce_fwd"),
    (r"skip_fwd_mfma_kernel<\d+, \d+, false", "pointwise_fwd"),
    (r"skip_bwd_mfma_kernel<\d+, \d+, true", "skip_reduce_bwd"),
    (r"skip_bwd_mfma_kernel<\d+, \d+, false", "pointwise_bwd"),
    # (first match wins: the skip fusion's instances before the pointwise ones)
    (r"pwbf_fwd_kernel<\d+, \d+, true, false, true>", "skip_reduce_fwd"),
    (r"pwbf_bwd_kernel<\d+, \d+, true, (true|false), true", "skip_reduce_bwd"),
    (r"pwbf_fwd_kernel", "pointwise_fwd"),
    (r"pwbf_bwd_kernel|pw_bwd_pf_kernel", "pointwise_bwd"),
    (r"conv3x3_fwd_kernel<\d+, \d+, \d+, false", "conv3x3_fwd"),
    (r"conv3x3_fwd_kernel<\d+, \d+, \d+, true", "conv3x3_dgrad"),
    (r"conv3x3_bf_fwd2?_kernel<\d+, \d+, \d+, false", "conv3x3_fwd_bf16"),
    (r"conv3x3_bf_fwd2_kernel<\d+, \d+, \d+, true", "conv3x3_dgrad_bf16"),
    (r"c3in3_bf16_wgrad_kernel<\d+, 2>", "stem_wgrad_bf16"),
    (r"c3in3_bf16_wgrad_kernel<\d+, 1>", "conv3x3_wgrad_guide"),
    (r"conv3x3_bf_fwd_kernel<\d+, \d+, \d+, true", "conv3x3_dgrad_bf16"),
    (r"conv3x3_bf_wgrad_kernel", "conv3x3_wgrad_bf16"),
    # the fixed-strip kernel under the three ids that launch it (csrc/conv3x3.hip):
    # 32-channel groups at stride 1 (conv3x3_wgrad), stride 2 (conv3x3s2_wgrad)
    (r"conv3x3_wgrad_wide_fixed_kernel<1, \d+, \d+, \d+, 32>", "conv3x3_wgrad"),
    (r"conv3x3_wgrad_wide_fixed_kernel<2,", "conv3x3s2_wgrad"),
    (r"conv3x3s2_wgrad_kernel", "conv3x3s2_wgrad"),
    (r"conv3x3_wgrad_wide\w*_kernel", "conv3x3_wgrad_wide"),
    (r"conv3x3_wgrad_kernel<3,", "conv3x3_wgrad_guide"),
    (r"conv3x3_wgrad_kernel", "conv3x3_wgrad"),
    (r"wgrad_reduce\w*_kernel", "conv3x3_wreduce"),
    (r"skip_fwd_kernel", "skip_reduce_fwd"),
    (r"skip_bwd_kernel", "skip_reduce_bwd"),
    (r"skip_slab_reduce_kernel<0>", "skip_reduce_bwd_reduce"),
    (r"skip_slab_reduce_kernel<1>", "pointwise_bwd"),
    (r"minmax_partial_kernel", "minmax"),
    (r"minmax_final_kernel", "minmax_final"),
    (r"depthnorm_kernel", "depthnorm_apply"),
    (r"ssim3_(l1|stream|pair)_kernel", "ssim3_l1"),
    (r"c1_mix_small_kernel<[^>]*false>", "conv1x1_fwd"),
    (r"c1_mix_small_kernel<[^>]*true>", "conv1x1_dgrad"),
    (r"cm_kernel<[^>]*false>", "conv1x1_fwd"),
    (r"cm_kernel<[^>]*true>", "conv1x1_dgrad"),
    (r"c1_wgrad(_small)?_kernel", "conv1x1_wgrad"),
    (r"c1_wreduce_kernel", "conv1x1_wreduce"),
    (r"c3s2_fwd_kernel", "conv3x3s2_fwd"),
    (r"c3s2_dgrad_kernel", "conv3x3s2_dgrad"),
    (r"c3s1_kernel<false", "conv3x3w_fwd"),
    (r"c3s1_kernel<true", "conv3x3w_dgrad"),
    # forward and data gradient run the same kernel: one combined key, which
    # bench.py apportions by the two ids' algorithmic bytes (same ratio)
    (r"wino_f23_kernel", "wino_fwd+wino_dgrad"),
    (r"wino_weight(2|_table)?_kernel", "wino_weight"),
    (r"bn_fwd_chan_kernel", "bn_fwd_apply_small"),
    (r"bn_bwd_chan_kernel", "bn_bwd_apply_small"),
    (r"dloss_final_kernel", "loss_final"),
    (r"dloss_map_kernel<1>", "depth_loss_bwd_coef"),
    (r"dloss_(fwd_stream|masked|map)_kernel", "depth_loss_fwd"),
    (r"dloss_(bwd_stream|masked_bwd|grad)_kernel", "depth_loss_bwd"),
    (r"loss_final_kernel", "loss_final"),
    (r"bn_stats_kernel", "bn_fwd_stats"),
    (r"bn_coef_kernel|bn_stats_merge_kernel", "bn_fwd_final"),
    (r"bn_apply_plane_kernel", "bn_fwd_apply"),
    (r"bn_apply_table_kernel", "bn_fwd_apply_small"),
    (r"bn_bwd_reduce_kernel", "bn_bwd_reduce"),
    (r"bn_bwd_apply_plane_kernel", "bn_bwd_apply"),
    (r"bn_bwd_apply_table_kernel", "bn_bwd_apply_small"),
    (r"skip_bwd_(reg|c1)_kernel", "skip_reduce_bwd"),
    (r"wattn_fwd_kernel", "window_attn_fwd"),
    (r"wattn_bwd_kernel", "window_attn_bwd"),
    (r"wattn_slab_reduce_kernel", "window_attn_bwd_reduce"),
    (r"dw_fwd_(strip|stream)_kernel", "dwconv_fwd"),
    (r"dw_bwd_(strip|stream)_kernel", "dwconv_bwd"),
    (r"dw_bwd_data_kernel", "dwconv_bwd_data"),
    (r"dw_bwd_weight_kernel", "dwconv_bwd_weight"),
    (r"dw_(wreduce|wsum)_kernel", "dwconv_wreduce"),
    (r"ln_fwd_kernel", "layernorm_fwd"),
    (r"ln_bwd_kernel", "layernorm_bwd"),
    (r"ln_wreduce_kernel", "layernorm_wreduce"),
    (r"transpose4?_kernel", "transpose"),
    (r"colsum_part_kernel<true>", "gelu_bwd_bias_grad"),
    (r"colsum_(part_kernel<false>|final_kernel)", "linear_bias_grad"),
    # forward and data gradient run the same kernel (as wino_f23_kernel)
    (r"convbf_fwd_(res_)?kernel", "convbf_fwd_bf16+convbf_dgrad_bf16"),
    (r"convbf_wgrad_kernel", "convbf_wgrad_bf16"),
    (r"convbf_wreduce_kernel", "convbf_wreduce"),
    (r"convbf_pack_(table_)?kernel", "convbf_pack"),
    (r"stem_bf16_fwd_kernel", "stem_fwd_bf16"),
    (r"stem_bf16_wgrad_kernel|stem_wreduce_kernel<0>", "stem_wgrad_bf16"),
    (r"stem_wreduce_kernel<1>", "conv3x3_wgrad_guide"),
    (r"stem_wreduce_kernel\(", "stem_wgrad_bf16"),  # builds before the tag
    (r"lin_wgrad_kernel", "linear_wgrad"),
    (r"lin_wreduce_kernel", "linear_wreduce"),
    (r"chansum_(part|final)_kernel", "conv_bias_grad"),
    (r"head_fwd_kernel", "head_conv_fwd"),
    (r"head_dgrad_kernel", "head_conv_dgrad"),
    (r"head_(wgrad|wreduce)_kernel", "head_conv_wgrad"),
    (r"eval_partial_kernel", "eval_sums"),
    (r"eval_final_kernel", "eval_final"),
    (r"nyu_augment_kernel", "nyu_augment"),
    # builds before round 5 (one untagged slab reduction for both callers)
    (r"skip_slab_reduce_kernel\(", "skip_reduce_bwd_reduce"),
]


def registry_name(sym: str):
    for pat, name in NAMES:
        if re.search(pat, sym):
            return name
    return None


def load(path, counter, last_steps):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "minmax_partial_kernel" in r["Kernel_Name"]]
    # exactly `last_steps` whole steps: from one step's minmax (the loss, mid-
    # step) to the same point `last_steps` steps later
    if len(marks) > last_steps:
        start, end = marks[-last_steps - 1], marks[-1]
    else:
        start, end = 0, len(rows)
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in rows[start:end]:
        name = registry_name(r["Kernel_Name"])
        if name:
            agg[name][0] += float(r["Counter_Value"])
            agg[name][1] += 1
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--last-steps", type=int, default=2)
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    f = load(a.fetch, "FETCH_SIZE", a.last_steps)
    w = load(a.write, "WRITE_SIZE", a.last_steps)
    out = {}
    for name in sorted(set(f) | set(w)):
        fk, fn = f.get(name, [0.0, 1])
        wk, wn = w.get(name, [0.0, 1])
        # per step too: the timing registry groups some helper launches under
        # the main kernel's name (e.g. a slab reduce), so ratios are taken per step
        out[name] = {"fetch_bytes_per_launch": 2 * fk * 1024 / fn,
                     "write_bytes_per_launch": wk * 1024 / wn,
                     "bytes_per_launch": 2 * fk * 1024 / fn + wk * 1024 / wn,
                     "bytes_per_step": (2 * fk + wk) * 1024 / a.last_steps,
                     "launches": fn}
    txt = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
