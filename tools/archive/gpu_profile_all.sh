#!/bin/bash
# Round profile: rocprofv3 kernel trace + stats of the cfg2 bench (and PMC
# FETCH/WRITE passes), then the cfg4 (newcrf) bench line and its trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMC=1 bash tools/gpu_profile.sh || exit $?
mkdir -p gpurun_out/prof_nc
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
echo "== newcrf bench ($(date +%T))"
timeout -k 10 600 python bench.py --workload newcrf --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/bench_newcrf.log 2>&1 || exit $?
tail -1 gpurun_out/bench_newcrf.log | cut -c1-300
echo "== newcrf trace ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_nc/trace" \
  -o r02 -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline \
  > gpurun_out/prof_nc/trace_bench.log 2>&1 || exit $?
echo done
