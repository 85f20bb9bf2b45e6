#!/bin/bash
# Round 6 AG: 64 / 128-row M tiles for padded wide 1x1s (MDE_C1_BM_AUTO) -- tests, cfg4 / cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ag}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_C1_BM_AUTO=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_mobilenet.py tests/test_gpu_newcrf.py tests/test_gpu_parity.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_C1_BM_AUTO=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nc_s$v.json 2> $OUT/bench_nc_s$v.log
  rc=$?; echo "bench nc small=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_nc_s$v.json'));k=b['hip_kernels'];print(b['value'], k['conv1x1_fwd']['ms_per_step'], k['conv1x1_dgrad']['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
for v in 0 1; do
  MDE_C1_BM_AUTO=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd_s$v.json 2> $OUT/bench_gd_s$v.log
  rc=$?; echo "bench gd small=$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_gd_s$v.json'));print(b['value'])")"; [ $rc -eq 0 ] || exit $rc
done
