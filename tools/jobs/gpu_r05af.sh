#!/bin/bash
# Round-5 call AF: skip fusion (reduce(relu(bn(r)) + d)) on bf16 products: tests, cfg3 step A/B (MDE_PW_BF).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_se_bn.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_PW_BF=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "pw_bf=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('skip') or n.startswith('pointwise')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
