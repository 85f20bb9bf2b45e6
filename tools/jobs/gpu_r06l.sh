#!/bin/bash
# Round 6 L: padded-channel 1x1 convs (MobileNetV3 off MIOpen) -- tests, cfg4 + cfg2 A/B, cfg4 trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06l}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_mobilenet.py tests/test_gpu_newcrf.py tests/test_gpu_sam.py tests/test_gpu_parity.py -x -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_C1_PAD=$v timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc_c$v.json 2> $OUT/bench_nc_c$v.log
  rc=$?; echo "bench nc c1pad=$v: $(head -c 200 $OUT/bench_nc_c$v.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd: $(head -c 200 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
MIOPEN_USER_DB_PATH=/tmp/mio_trace/db MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_trace/cache \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$OUT/trace_nc" -o r06 -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
