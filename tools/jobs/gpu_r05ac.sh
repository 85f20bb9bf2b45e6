#!/bin/bash
# Round-5 call AC: conv3x3 bf16 tile height A/B with the 16-byte row stage (MDE_BF_RPW=1 / 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ac
mkdir -p $OUT
export TMPDIR=/tmp
for v in 1 2; do
  MDE_BF_RPW=$v timeout -k 10 200 python3 -u tools/kbench.py --only convbf > $OUT/kb_$v.log 2>&1; rc=$?; echo "rpw=$v"; grep "HIP" $OUT/kb_$v.log; [ $rc -eq 0 ] || exit $rc
done
