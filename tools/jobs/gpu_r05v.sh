#!/bin/bash
# Round-5 call V: conv3x3 bf16 forward / data gradient with the row stage (conv3x3_bf_fwd2_kernel, MDE_C3BF_V2 A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_C3BF_V2=$v timeout -k 10 200 python3 -u tools/kbench.py --only convbf > $OUT/kb_$v.log 2>&1; rc=$?; echo "v2=$v"; grep "HIP" $OUT/kb_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if 'conv3x3' in n])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
