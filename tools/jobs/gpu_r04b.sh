#!/bin/bash
# Round-4 call B: the full GPU suite (RCCL cases in child processes), then the
# captured-RCCL test in the pytest process itself (as in the two recorded
# aborts of round 3), after the file's other graph tests, with HIP error
# logging; then call C (conv maps, NHWC A/B, wide-wgrad A/B + PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04b
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -n 6 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
AMD_LOG_LEVEL=1 MDE_RCCL_INPROC=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_graph.py -x -v \
  --timeout 400 --timeout-method thread > $OUT/inproc.log 2>&1
rc=$?
echo "inproc rc=$rc"
grep -v "NCCL INFO\|Cannot find the function" $OUT/inproc.log | tail -n 30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04c.sh
