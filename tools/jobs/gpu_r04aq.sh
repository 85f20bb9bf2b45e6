#!/bin/bash
# Round-4 call AQ: rocprofv3 kernel traces of the cfg3 (bf16) and cfg4 steps at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04aq
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd_bf16" -o r04 \
  -- python3 bench.py --amp bf16 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_gd_bf16.log 2>&1
rc=$?; echo "trace bf16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_nc" -o r04 \
  -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace nc rc=$rc"
