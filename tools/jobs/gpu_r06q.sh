#!/bin/bash
# Round 6 Q: residual adds fused into the NewCRF LayerNorms -- tests, cfg4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06q}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_newcrf.py tests/test_gpu_sam.py tests/test_gpu_graph.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_LN_ADD=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc_l$v.json 2> $OUT/bench_nc_l$v.log
  rc=$?; echo "bench nc lnadd=$v: $(head -c 200 $OUT/bench_nc_l$v.json)"; [ $rc -eq 0 ] || exit $rc
done
