#!/bin/bash
# Round-5 call AM: guide convs' statistics epilogue without per-pixel bounds
# tests on whole row segments, hardware bf16 rounding: tests, timing, VALU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R05_OUT:-r05am}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/guide_bench.py 2>&1 | grep guide && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES" TAG=guide_d ARGS="tools/guide_bench.py --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-400 || exit 1
for amp in fp32 bf16; do
  timeout -k 10 300 python3 -u bench.py --amp $amp --no-cpu-baseline --steps 30 --warmup 5 > $OUT/bench_$amp.json 2> $OUT/bench_$amp.log
  rc=$?; echo "bench $amp rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$amp.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step'], k[n].get('GBps')) for n in k if n.startswith('conv3x3_fwd')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
