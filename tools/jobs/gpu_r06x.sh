#!/bin/bash
# Round 6 X: cfg4 op attribution (current tree).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06x}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload newcrf --bs 16 --top 40 > $OUT/aten_nc.log 2>&1
rc=$?; echo "aten nc rc=$rc"; exit $rc
