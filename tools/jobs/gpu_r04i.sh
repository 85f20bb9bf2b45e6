#!/bin/bash
# Round-4 call I: bf16 guide-conv tests + graph tests, the cfg2 bench line,
# the cfg3 (bf16) A/B of the bf16 guide convs, and a rocprofv3 kernel trace
# of the cfg2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_resume.py \
  -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -v "Cannot find the function" $OUT/tests.log | tail -n 20 | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench rc=$rc"; head -c 600 $OUT/bench_gd.json; echo; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  MDE_GUIDE_BF16=$v timeout -k 10 300 python3 -u bench.py --amp bf16 --steps 30 --warmup 10 --no-cpu-baseline \
    --no-kernel-timing > $OUT/ab_bf16_$v.json 2> $OUT/ab_bf16_$v.log
  rc=$?; echo "GUIDE_BF16=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_bf16_$v.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd" -o r04 \
  -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_gd.log 2>&1
rc=$?; echo "trace rc=$rc"
