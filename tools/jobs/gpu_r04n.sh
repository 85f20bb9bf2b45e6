#!/bin/bash
# Round-4 call N: (1) bisect the bf16 GuideDepth golden-test regression over
# this session's switches (guide bf16 convs, one-launch small BN, two-column
# SSIM); (2) the persistent Winograd kernels: tests and per-shape timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
T=tests/test_gpu_bf16.py::test_guidedepth_bf16_golden_vs_float64_oracle
for cfg in "MDE_NONE=1" "MDE_GUIDE_BF16=0" "MDE_BN_CHAN=0" "MDE_SSIM_PAIR=0" "MDE_GUIDE_BF16=0 MDE_BN_CHAN=0 MDE_SSIM_PAIR=0"; do
  env $cfg timeout -k 10 300 python3 -u -m pytest $T -q -s --timeout 240 --timeout-method thread > $OUT/bisect.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -o 'HIP bf16 {[^}]*}' $OUT/bisect.log | head -1)"
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "wino tests rc=$rc"; tail -n 5 $OUT/tests.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/c1_bench.py > $OUT/c1_bench.txt 2>&1
rc=$?; grep "3x3s1" $OUT/c1_bench.txt | cut -c1-300; exit $rc
