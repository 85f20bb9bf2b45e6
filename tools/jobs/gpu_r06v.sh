#!/bin/bash
# Round 6 V: GEMM table -- its test, cfg3 and SAM A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06v}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_linear.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  for wl in "sam" "guidedepth --amp bf16"; do
    tag=$(echo $wl | tr -d ' -')
    MDE_GEMM_TABLE=$v timeout -k 10 300 python3 -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_${tag}_t$v.json 2> $OUT/bench_${tag}_t$v.log
    rc=$?; echo "bench $tag table=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_${tag}_t$v.json'));print(b['value'], b['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
