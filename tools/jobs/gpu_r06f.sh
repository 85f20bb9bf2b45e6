#!/bin/bash
# Round 6 F: 16 -> 16 full-resolution conv, RPW 1 vs 2 (MDE_C3_VARIANT), kernel + cfg2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06f}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for v in 0 1; do
  MDE_C3_VARIANT=$v timeout -k 10 200 python3 -u tools/guide_bench.py --cin16 > $OUT/c16_v$v.log 2>&1
  rc=$?; echo "variant $v"; grep guide $OUT/c16_v$v.log; [ $rc -eq 0 ] || exit $rc
done
MDE_C3_VARIANT=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_parity.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_v1.log 2>&1
rc=$?; echo "tests v1 rc=$rc"; tail -1 $OUT/tests_v1.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_C3_VARIANT=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_v$v.json 2> $OUT/bench_v$v.log
  rc=$?; echo "bench v=$v: $(head -c 160 $OUT/bench_v$v.json)"; [ $rc -eq 0 ] || exit $rc
done
