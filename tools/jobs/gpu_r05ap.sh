#!/bin/bash
# Round-5 call AP: statistics epilogues of the bf16 3x3 forward and the
# resident convbf forward without per-pixel tests on whole tiles: tests, cfg3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ap
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_convbf.py tests/test_gpu_conv3x3.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --amp bf16 --no-cpu-baseline --steps 30 --warmup 5 > $OUT/bench_bf16_$i.json 2> $OUT/bench_bf16_$i.log
  rc=$?; echo "bench bf16 rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16_$i.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('conv')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
