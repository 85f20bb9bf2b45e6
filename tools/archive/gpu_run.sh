#!/bin/bash
# Generic GPU-box wrapper: repo MIOpen cache, a heartbeat under gpurun_out/
# (MIOpen's first-use compiles can be silent for minutes), the MIOpen cache
# handed back in gpurun_out/miopen_sync, and a time limit on the command.
#   bash tools/gpu_run.sh SECONDS LOGNAME cmd...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db
( while sleep 60; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "rc=$rc"; tail -n 5 "gpurun_out/$log"
exit $rc
