#!/bin/bash
# Round-4 call J: parity of this session's kernels (stride-2 forward 2D tiles +
# 3-channel stem, one-block-per-channel small BN, SE backward tail launch,
# sliced weight-gradient reduction, two-column SSIM), then their A/Bs:
# weight-gradient passes per shape (MDE_WRED_SLICES=1 vs auto), SSIM
# (MDE_SSIM_PAIR 0/1, MDE_SSIM_ORDER, waves), stride-2 per-shape timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_conv3x3s2.py tests/test_gpu_bn.py tests/test_gpu_se_bn.py \
  tests/test_gpu_parity.py tests/test_gpu_conv3x3.py tests/test_gpu_bf16.py tests/test_gpu_resume.py \
  -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -v "Cannot find the function" $OUT/tests.log | tail -n 25 | cut -c1-300
[ $rc -le 1 ] || exit $rc
for v in 1 0; do
  MDE_WRED_SLICES=$v timeout -k 10 300 python3 -u tools/wred_bench.py > $OUT/wred_$v.txt 2>&1
  rc=$?; tail -n 1 $OUT/wred_$v.txt; [ $rc -eq 0 ] || exit $rc
done
for cfg in "MDE_SSIM_PAIR=0" "MDE_SSIM_PAIR=0 MDE_SSIM_ORDER=1" "MDE_SSIM_PAIR=0 MDE_SSIM_ORDER=2" \
           "MDE_SSIM_PAIR=1" "MDE_SSIM_PAIR=1 MDE_SSIM_WAVES=5632" "MDE_SSIM_PAIR=1 MDE_SSIM_WAVES=4224"; do
  env $cfg timeout -k 10 300 python3 -u tools/kbench.py --only loss > $OUT/ssim.txt 2>&1
  rc=$?; echo "$cfg: $(grep ssim3 $OUT/ssim.txt | head -2 | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u tools/c1_bench.py > $OUT/c1_bench.txt 2>&1
rc=$?; grep "3x3s2\|per cfg2" $OUT/c1_bench.txt; [ $rc -eq 0 ] || exit $rc
