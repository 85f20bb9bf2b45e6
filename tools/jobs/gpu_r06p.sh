#!/bin/bash
# Round 6 P: head conv (head.hip) + biased 1x1 bridge on HIP -- tests, cfg4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06p}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_head.py tests/test_gpu_newcrf.py tests/test_gpu_conv1x1.py tests/test_gpu_sam.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_HEAD_CONV=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc_h$v.json 2> $OUT/bench_nc_h$v.log
  rc=$?; echo "bench nc head=$v: $(head -c 200 $OUT/bench_nc_h$v.json)"; [ $rc -eq 0 ] || exit $rc
done
