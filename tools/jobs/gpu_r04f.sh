#!/bin/bash
# Round-4 call F: the new wide 1x1 and stride-2 3x3 kernels -- parity tests
# first (each under its own limit), per-shape bench vs MIOpen, then the cfg2
# step A/B (new kernels on vs MDE_C1_WIDE=0 MDE_S2_FWD=0, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_conv3x3s2.py -v \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $OUT/tests.log | tail -n 40 | cut -c1-200
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u tools/c1_bench.py > $OUT/c1_bench.log 2>&1
rc=$?; grep "1x1\|3x3s\|step" $OUT/c1_bench.log; [ $rc -eq 0 ] || exit $rc
for v in on s1off off on s1off off; do
  case $v in on) e="A=1";; s1off) e="MDE_C3_WIDE=0";; off) e="MDE_C1_WIDE=0 MDE_S2_FWD=0 MDE_C3_WIDE=0";; esac
  env $e timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline \
    --no-kernel-timing > $OUT/ab_$v.json 2> $OUT/ab_$v.log
  rc=$?; echo "$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$v.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
