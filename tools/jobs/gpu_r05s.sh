#!/bin/bash
# Round-5 call S: 32 -> 32 at 120x160 (DDRNet layer1): conv3x3 bf16 kernel vs convbf.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/convbf_bench.py --only 32,32,120,160,3,1 > $OUT/cbf.log 2>&1; rc=$?; grep "(32" $OUT/cbf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/kbench.py --only convbf > $OUT/kb.log 2>&1; rc=$?; grep "HIP" $OUT/kb.log; [ $rc -eq 0 ] || exit $rc
