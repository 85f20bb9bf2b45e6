#!/bin/bash
# Round-4 call E: the wide 1x1 conv kernels -- parity tests, per-shape bench vs
# MIOpen, and the cfg2 step A/B (MDE_C1_WIDE=1 vs 0, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/c1_bench.py > $OUT/c1_bench.log 2>&1
rc=$?; grep "1x1\|per cfg2" $OUT/c1_bench.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  MDE_C1_WIDE=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline \
    --no-kernel-timing > $OUT/ab_$v.json 2> $OUT/ab_$v.log
  rc=$?; echo "MDE_C1_WIDE=$v rc=$rc $(head -c 140 $OUT/ab_$v.json | cut -c100-140)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -n 5 $OUT/suite.log
