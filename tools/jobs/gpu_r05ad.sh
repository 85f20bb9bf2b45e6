#!/bin/bash
# Round-5 call AD: 32-channel conv3x3 bf16 tile heights + bf16 BN forward apply with 4 images a block (MDE_BN_IPB A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_bn.py tests/test_gpu_bf16.py tests/test_gpu_convbf.py tests/test_gpu_conv3x3.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for v in 4 1; do
  MDE_BN_IPB=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "ipb=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('bn_fwd') or n.startswith('conv3x3')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
