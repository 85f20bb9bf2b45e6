#!/bin/bash
# Round-5 call N: convbf parity + per-shape timing + the cfg3 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/convbf.log 2>&1
rc=$?; echo "convbf rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/convbf.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids $OUT/kbench.log | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_bf16.json 2> $OUT/bench_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; exit $rc
