#!/bin/bash
# Round 6 C: Winograd lane-contiguous U layout -- tests, per-shape timing, cfg2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/wino_tests.log 2>&1
rc=$?; echo "wino tests rc=$rc"; tail -2 $OUT/wino_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/wino_bench.py --modes 2,6 > $OUT/wino_bench.log 2>&1
rc=$?; grep wino $OUT/wino_bench.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do
  MDE_WINO_X=$x timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_x$x.json 2> $OUT/bench_x$x.log
  rc=$?; echo "bench X=$x: $(head -c 200 $OUT/bench_x$x.json)"; [ $rc -eq 0 ] || exit $rc
done
