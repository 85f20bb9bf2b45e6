#!/bin/bash
# Round 6: the whole GPU suite (one process), smoke(), then the cfg2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06a}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -8 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 30 --warmup 5 > $OUT/bench_gd_fp32.json 2> $OUT/bench_gd_fp32.log
rc=$?; head -c 400 $OUT/bench_gd_fp32.json; echo; exit $rc
