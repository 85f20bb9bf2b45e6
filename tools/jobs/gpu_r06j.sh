#!/bin/bash
# Round 6 J: cfg4 after the Linear weight gradient -- bench (kernel timing) + steady-state trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06j}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc: $(head -c 200 $OUT/bench_nc.json)"; [ $rc -eq 0 ] || exit $rc
MIOPEN_USER_DB_PATH=/tmp/mio_trace/db MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_trace/cache \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$OUT/trace_nc" -o r06 -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
