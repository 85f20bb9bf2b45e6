#!/bin/bash
# Round-4 call Y2: the watchdog / capture stream rules (eager collectives
# never on a captured stream, thread-local capture): both RCCL children
# directly with step markers, then the graph / DP test files.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04y
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 AMD_LOG_LEVEL=1 NCCL_DEBUG=WARN
for m in overlap flat; do
  MDE_RCCL_TRACE=1 MASTER_PORT=29533 timeout -k 10 300 python3 -u tests/_rccl_graph_child.py $m > $OUT/child_$m.log 2>&1
  rc=$?; echo "child $m rc=$rc"; grep -v "Cannot find the function" $OUT/child_$m.log | grep -E "probe|OK|rror|what|nodes" | head -12 | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_graph.py tests/test_gpu_graph_dp.py -q -rfE \
  -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/graph.log 2>&1
rc=$?; echo "graph tests rc=$rc"; grep -v "Cannot find the function" $OUT/graph.log | grep -E "^FAILED|^ERROR|passed|failed" | tail -n 10 | cut -c1-300
