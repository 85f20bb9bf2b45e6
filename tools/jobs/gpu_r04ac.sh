#!/bin/bash
# Round-4 call AC: x2 resize kernels with branch-free edge loads: parity,
# kbench resize at MDE_X2_QUAD=1 (fp32 fwd on the pair kernel) and 2 (quad for
# both), cfg3 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ac
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider \
  -k "bilinear or resize or nearest or guidedepth" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 12 | cut -c1-300; [ $rc -le 1 ] || exit $rc
for q in 1 2; do
  MDE_X2_QUAD=$q timeout -k 10 300 python3 -u tools/kbench.py --only resize > $OUT/kbench_resize_q$q.txt 2>&1
  rc=$?; echo "MDE_X2_QUAD=$q"; grep "x2" $OUT/kbench_resize_q$q.txt | cut -c1-90; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 -u bench.py --amp bf16 --no-cpu-baseline > $OUT/bench_gd_bf16.json 2> $OUT/bench_gd_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(head -c 200 $OUT/bench_gd_bf16.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd_bf16.json'));print(d['path_roofline']);print({k:v for k,v in d['hip_kernels'].items() if 'bilinear' in k or 'nearest' in k})"
