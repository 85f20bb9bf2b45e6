#!/bin/bash
# Round-4 call M: the Winograd stride-1 convs in the cfg2 step (MDE_WINO A/B,
# interleaved), the GuideDepth parity / graph tests with Winograd on, and the
# cfg2 bench line with Winograd on (per-kernel times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_WINO=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_parity.py tests/test_gpu_resume.py \
  -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests (WINO=1) rc=$rc"; grep -v "Cannot find the function" $OUT/tests.log | tail -n 15 | cut -c1-300
[ $rc -le 1 ] || exit $rc
for v in 0 1 0 1; do
  MDE_WINO=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_wino_$v.json 2> $OUT/ab_wino_$v.log
  rc=$?; echo "WINO=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_wino_$v.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
MDE_WINO=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_wino.json 2> $OUT/bench_wino.log
rc=$?; python3 -c "import json;d=json.load(open('$OUT/bench_wino.json'));k=d['hip_kernels'];print(d['value'],{n:(v['ms_per_step'],v.get('TFLOPs')) for n,v in k.items() if 'wino' in n or 'conv3x3' in n})"; exit $rc
