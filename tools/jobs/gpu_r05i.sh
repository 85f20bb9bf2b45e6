#!/bin/bash
# Round-5 call I: the bf16 stem kernels (parity), the bf16 model tests, cfg3
# bench + steady-state kernel trace (MIOpen's transposes should be gone).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stem.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/stem.log 2>&1
rc=$?; echo "stem rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|Error" $OUT/stem.log | tail -8 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/models.log 2>&1
rc=$?; echo "models rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/models.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_bf16.json 2> $OUT/bench_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd_bf16" -o r05 -- python3 bench.py --amp bf16 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
