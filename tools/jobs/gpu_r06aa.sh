#!/bin/bash
# Round 6 AA: cfg3 op attribution (elementwise leftovers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06aa}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload guidedepth --bs 32 --amp bf16 --top 40 > $OUT/aten_gd_bf16.log 2>&1
rc=$?; echo "aten rc=$rc"; exit $rc
