#!/bin/bash
# Round-4 call X: the RCCL capture tests with thread-local capture (the
# watchdog-query abort of r04w), then the graph / DP tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04x
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
AMD_LOG_LEVEL=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_graph.py tests/test_gpu_graph_dp.py -q -rfE \
  -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/graph.log 2>&1
rc=$?; echo "graph tests rc=$rc"; grep -v "Cannot find the function" $OUT/graph.log | grep -E "^FAILED|^ERROR|passed|failed|Error|what" | tail -n 25 | cut -c1-300
