#!/bin/bash
# Round-5 call P: convbf + bf16 model tests, cfg3 bench with / without the one-launch filter pack.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_convbf.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_wino.py tests/test_gpu_newcrf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_CONVBF_PACK_ALL=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "pack_all=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'], d['ms_per_step'], d['hip_kernels'].get('convbf_pack'))" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
