#!/bin/bash
# Round 6 K: padded-input-channel wide weight gradients (the NewCRF projections off MIOpen) -- tests, cfg4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06k}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_wino.py tests/test_gpu_newcrf.py tests/test_gpu_linear.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_WIDE_PAD=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc_p$v.json 2> $OUT/bench_nc_p$v.log
  rc=$?; echo "bench nc pad=$v: $(head -c 200 $OUT/bench_nc_p$v.json)"; [ $rc -eq 0 ] || exit $rc
done
