#!/bin/bash
# Round-5 call A: the data-parallel changes (no per-step BN broadcast,
# sync_buffers on close) on the GPU: graph / DP tests, then a short cfg2
# bench line through the new bench.py main.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_graph_dp.py tests/test_gpu_graph.py -q -rfE \
  -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|no tests ran" $OUT/tests.log | tail -n 8 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 300 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
