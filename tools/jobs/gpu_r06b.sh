#!/bin/bash
# Round 6 B: Winograd persistent kernel -- bitwise test, per-shape A/B, then the graph / DP tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/wino_tests.log 2>&1
rc=$?; echo "wino tests rc=$rc"; tail -3 $OUT/wino_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/wino_bench.py --modes 0,1 > $OUT/wino_bench.log 2>&1
rc=$?; grep wino $OUT/wino_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_graph.py tests/test_gpu_graph_dp.py tests/test_gpu_parity.py tests/test_gpu_convbf.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/graph_tests.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -3 $OUT/graph_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  MDE_WINO_P=$m timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_p$m.json 2> $OUT/bench_p$m.log
  rc=$?; echo "bench P=$m: $(head -c 200 $OUT/bench_p$m.json)"; [ $rc -eq 0 ] || exit $rc
done
