#!/bin/bash
# Round 6 N: cfg2 op attribution (which convs still reach MIOpen / rocBLAS, elementwise ops).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06n}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload guidedepth --bs 32 --top 40 > $OUT/aten_gd.log 2>&1
rc=$?; echo "aten gd rc=$rc"; exit $rc
