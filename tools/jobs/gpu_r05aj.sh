#!/bin/bash
# Round-5 call AJ: feasibility timing for split-bf16 fp32 convolutions (next
# round): the bf16 implicit-GEMM kernels at 3x the input channels (forward /
# data gradient: [x_hi, x_hi, x_lo] against [w_hi, w_lo, w_hi]) and at 3x the
# batch (weight gradient: [x_hi; x_hi; x_lo] against [g_hi; g_lo; g_hi]),
# beside the fp32 Winograd forward of the same convs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/wino_bench.py > $OUT/wino.log 2>&1; rc=$?; grep wino $OUT/wino.log; [ $rc -eq 0 ] || exit $rc
for s in 96,32,120,160,3,1 192,64,60,80,3,1 384,128,30,40,3,1 768,256,15,20,3,1; do
  timeout -k 10 120 python3 -u tools/convbf_bench.py --only $s > $OUT/cbf_$s.log 2>&1; rc=$?; grep "^(" $OUT/cbf_$s.log; [ $rc -eq 0 ] || exit $rc
done
for s in 32,32,120,160,3,1 64,64,60,80,3,1 128,128,30,40,3,1 256,256,15,20,3,1; do
  timeout -k 10 120 python3 -u tools/convbf_bench.py --n 96 --only $s > $OUT/cbfw_$s.log 2>&1; rc=$?; grep "^(" $OUT/cbfw_$s.log; [ $rc -eq 0 ] || exit $rc
done
