#!/bin/bash
# Round 6 Y: stride-1 1x1 forward on HIP for off-grid channel counts (MDE_C1_FWD) -- tests, cfg4 / cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06y}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_mobilenet.py tests/test_gpu_newcrf.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in none pad none pad all; do
  MDE_C1_FWD=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc_$v.json 2> $OUT/bench_nc_$v.log
  rc=$?; echo "bench nc c1fwd=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_nc_$v.json'));print(b['value'], b['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
for v in pad all; do
  MDE_C1_FWD=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd_$v.json 2> $OUT/bench_gd_$v.log
  rc=$?; echo "bench gd c1fwd=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_gd_$v.json'));print(b['value'], b['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
