#!/bin/bash
# rocprofv3 kernel trace of bench steps per workload -> gpurun_out/trace_<wl>/ ; WORKLOADS="gd_fp32 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out .miopen/cache .miopen/db
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=$ROOT/.miopen/cache MIOPEN_USER_DB_PATH=$ROOT/.miopen/db
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
for wl in ${WORKLOADS:-gd_fp32}; do
  case $wl in
    gd_fp32) args="--workload guidedepth" ;;
    gd_bf16) args="--workload guidedepth --amp bf16" ;;
    nc_fp32) args="--workload newcrf" ;;
    nc_bf16) args="--workload newcrf --amp bf16" ;;
  esac
  echo "== trace $wl ($(date +%T))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/trace_$wl" \
      -o r03 -- python3 bench.py $args --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing \
      > gpurun_out/trace_$wl.log 2>&1
  rc=$?; tail -n 1 gpurun_out/trace_$wl.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
