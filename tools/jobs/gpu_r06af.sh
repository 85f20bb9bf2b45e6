#!/bin/bash
# Round 6 AF: 16->16 full-resolution 3x3 weight gradient at three blocks a CU (MDE_C3_VARIANT=3) -- tests, kbench, cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06af}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_C3_VARIANT=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv3x3.py -k "wgrad" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_v3.log 2>&1
rc=$?; echo "tests v3 rc=$rc $(tail -1 $OUT/tests_v3.log)"; [ $rc -eq 0 ] || exit $rc
for v in 0 3 0 3; do
  MDE_C3_VARIANT=$v timeout -k 10 120 python3 -u tools/wgrad_bench.py --only 32,16,16,480,640 > $OUT/wb_v$v.txt 2>&1
  rc=$?; echo "wgrad_bench v$v: $(tail -2 $OUT/wb_v$v.txt | head -1)"; [ $rc -eq 0 ] || exit $rc
done
for v in 0 3 0 3; do
  MDE_C3_VARIANT=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_gd_v$v.json 2> $OUT/bench_gd_v$v.log
  rc=$?; echo "bench gd v$v: $(python3 -c "import json;b=json.load(open('$OUT/bench_gd_v$v.json'));k=b['hip_kernels'];print(b['value'], k['conv3x3_wgrad']['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
