#!/bin/bash
# Round-4 call G: wide-conv kernels after the division fix -- parity tests,
# per-shape bench, cfg2 A/B (HIP 1x1 + stride-2 vs MIOpen, interleaved), then
# the full GPU suite (HIP error log on for the RCCL child).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_conv3x3s2.py -q \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 15 $OUT/tests.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u tools/c1_bench.py > $OUT/c1_bench.log 2>&1
rc=$?; grep "1x1\|3x3s\|step" $OUT/c1_bench.log; [ $rc -eq 0 ] || exit $rc
for v in on off on off; do
  case $v in on) e="A=1";; off) e="MDE_C1_WIDE=0 MDE_S2_FWD=0";; esac
  env $e timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline \
    --no-kernel-timing > $OUT/ab_$v.json 2> $OUT/ab_$v.log
  rc=$?; echo "$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$v.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -v "Cannot find the function" $OUT/suite.log | tail -n 30 | cut -c1-400
