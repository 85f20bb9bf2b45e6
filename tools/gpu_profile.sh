#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (separate PMC passes when PMC=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$ROOT/.miopen/cache
export MIOPEN_USER_DB_PATH=$ROOT/.miopen/db
mkdir -p "$MIOPEN_CUSTOM_CACHE_DIR" "$MIOPEN_USER_DB_PATH"
( while sleep 60; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
STEPS=${STEPS:-5}
WARMUP=${WARMUP:-3}
TAG=${TAG:-r02}
echo "== trace ($(date +%T))"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$ROOT/gpurun_out/prof/trace" -o "$TAG" -- \
  python3 "$ROOT/bench.py" --steps "$STEPS" --warmup "$WARMUP" --no-cpu-baseline ${BENCH_ARGS:-} \
  > gpurun_out/prof/trace_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -n 5 gpurun_out/prof/trace_bench.log; [ $rc -eq 0 ] || exit $rc
if [ "${PMC:-0}" = 1 ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $ctr ($(date +%T))"
    timeout -k 10 900 rocprofv3 --pmc "$ctr" --output-format csv \
      -d "$ROOT/gpurun_out/prof/pmc_$ctr" -o "$TAG" -- \
      python3 "$ROOT/bench.py" --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing ${BENCH_ARGS:-} \
      > "gpurun_out/prof/pmc_$ctr.log" 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"; tail -n 3 "gpurun_out/prof/pmc_$ctr.log"; [ $rc -eq 0 ] || exit $rc
  done
fi
find gpurun_out/prof -name "*.csv" | head -20
