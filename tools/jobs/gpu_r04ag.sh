#!/bin/bash
# Round-4 call AG: 64-channel Winograd with a double-buffered raw tile (two
# barriers per chunk): wino parity, per-shape timing, cfg2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ag
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 8 | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/wino_bench.py > $OUT/wino.txt 2>&1
rc=$?; cat $OUT/wino.txt | tail -n 8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 200 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd.json'));print({k:v for k,v in d['hip_kernels'].items() if 'wino' in k})"
