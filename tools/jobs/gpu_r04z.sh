#!/bin/bash
# Round-4 call Z: bf16 storage for every bilinear ratio, the fused nearest
# guide pyramid: parity tests, resize kbench, cfg3 and cfg2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04z
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -rfE -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 12 | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/kbench.py --only resize > $OUT/kbench_resize.txt 2>&1
rc=$?; cat $OUT/kbench_resize.txt | grep -v "^\s*$" | tail -n 20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --amp bf16 > $OUT/bench_gd_bf16.json 2> $OUT/bench_gd_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(head -c 200 $OUT/bench_gd_bf16.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd_bf16.json'));print(d['path_roofline']);print({k:v for k,v in d['hip_kernels'].items() if 'bilinear' in k or 'nearest' in k})"
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 200 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd.json'));print(d['path_roofline'])"
