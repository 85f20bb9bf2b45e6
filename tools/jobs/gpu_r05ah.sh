#!/bin/bash
# Round-5 call AH: Winograd 32-channel blocks at three a CU: kernels + cfg2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -3 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/wino_bench.py 2>&1 | grep wino
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('wino')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
