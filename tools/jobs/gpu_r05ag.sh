#!/bin/bash
# Round-5 call AG: the prefetching pointwise backward on fp32 operands (16 -> 8 / 16 -> 16): tests, kernels, cfg2 step A/B (MDE_PW_PF).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_graph.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_PW_PF=$v timeout -k 10 200 python3 -u tools/pw_bf16_bench.py --dtype fp32 > $OUT/pw_$v.log 2>&1; rc=$?; echo "pf=$v"; grep "pointwise_bwd" $OUT/pw_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 1 0; do
  MDE_PW_PF=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "pf=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('pointwise')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
