#!/bin/bash
# Round 6 G: the one-launch Winograd filter-transform table -- tests, cfg2 A/B (MDE_WINO_TABLE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06g}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_resume.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_WINO_TABLE=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_t$v.json 2> $OUT/bench_t$v.log
  rc=$?; echo "bench table=$v: $(head -c 160 $OUT/bench_t$v.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload newcrf --bs 16 --top 30 > $OUT/aten_nc.log 2>&1
rc=$?; echo "aten nc rc=$rc"; exit $rc
