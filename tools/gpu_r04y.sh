#!/bin/bash
# Round-4 call Y: where does the watchdog query a captured event?  The
# overlap child with step markers, the watchdog logging CUDA errors instead of
# rethrowing them (no abort), then the same with the event cache off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04y
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MDE_RCCL_TRACE=1 AMD_LOG_LEVEL=1 NCCL_DEBUG=WARN
MASTER_PORT=29531 TORCH_NCCL_RETHROW_CUDA_ERRORS=0 timeout -k 10 300 python3 -u tests/_rccl_graph_child.py overlap \
  > $OUT/child_norethrow.log 2>&1
rc=$?; echo "norethrow rc=$rc"; grep -v "Cannot find the function" $OUT/child_norethrow.log | grep -E "step|probe|OK|rror|what|graph" | head -40 | cut -c1-250
[ $rc -eq 0 ] || exit $rc
MASTER_PORT=29532 TORCH_NCCL_CUDA_EVENT_CACHE=0 timeout -k 10 300 python3 -u tests/_rccl_graph_child.py overlap \
  > $OUT/child_nocache.log 2>&1
rc=$?; echo "nocache rc=$rc"; grep -v "Cannot find the function" $OUT/child_nocache.log | grep -E "step|probe|OK|rror|what|graph" | head -40 | cut -c1-250
