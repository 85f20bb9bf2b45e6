#!/bin/bash
# Round 6 D: relu folds + residual-gradient slot -- targeted tests, then the whole suite, then cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06d}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resume.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/targeted.log 2>&1
rc=$?; echo "targeted rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/targeted.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MDE_RES_SLOT=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_slot$v.json 2> $OUT/bench_slot$v.log
  rc=$?; echo "bench slot=$v: $(head -c 200 $OUT/bench_slot$v.json)"; [ $rc -eq 0 ] || exit $rc
done
