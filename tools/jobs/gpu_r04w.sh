#!/bin/bash
# Round-4 call W: the full GPU suite at HEAD (one-launch Winograd weight
# transforms, adaptive wide-wgrad blocks, per-channel bf16 tile height), then
# the cfg2 / cfg3 (bf16) / cfg4 bench lines and a rocprofv3 kernel trace of cfg2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04w
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
AMD_LOG_LEVEL=1 timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -v "Cannot find the function" $OUT/suite.log | grep -E "^FAILED|^ERROR|passed|failed" | tail -n 25 | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 300 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --amp bf16 > $OUT/bench_gd_bf16.json 2> $OUT/bench_gd_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(head -c 300 $OUT/bench_gd_bf16.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --workload newcrf > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc rc=$rc $(head -c 300 $OUT/bench_nc.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd" -o r04 \
  -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_gd.log 2>&1
rc=$?; echo "trace rc=$rc"
