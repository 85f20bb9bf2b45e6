#!/bin/bash
# Round 6 Z: float4 transpose -- tests, cfg4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06z}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_newcrf.py tests/test_gpu_sam.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_TRANSPOSE4=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nc_t$v.json 2> $OUT/bench_nc_t$v.log
  rc=$?; echo "bench nc t4=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_nc_t$v.json'));print(b['value'], b['ms_per_step'], b['hip_kernels']['transpose'])")"; [ $rc -eq 0 ] || exit $rc
done
