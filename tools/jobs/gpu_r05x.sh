#!/bin/bash
# Round-5 call X: fp32 conv3x3 (and bf16-output guide convs) with the LDS-staged output tile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_graph.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/kbench.py --only conv > $OUT/kb.log 2>&1; rc=$?; grep "HIP" $OUT/kb.log; [ $rc -eq 0 ] || exit $rc
for a in fp32 bf16; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp $a --steps 30 --warmup 5 > $OUT/bench_$a.json 2> $OUT/bench_$a.log
  rc=$?; echo "bench $a rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$a.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('conv3x3')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
