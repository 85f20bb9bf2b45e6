#!/bin/bash
# Round-4 call AD: NewCRF projections (3x3 + bias) on the HIP Winograd path:
# wino + NewCRF / SAM parity, cfg4 bench line + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04ad
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_newcrf.py tests/test_gpu_sam.py -q -rfE \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 12 | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --workload newcrf > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc rc=$rc $(head -c 200 $OUT/bench_nc.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_nc.json'));print(d['roofline']);print({k:v for k,v in d['hip_kernels'].items() if 'wino' in k})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_nc" -o r04 \
  -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace rc=$rc"
