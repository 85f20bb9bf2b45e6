#!/bin/bash
# Round 6 AI: 1x1 channel-mix accuracy vs float64, cm_kernel vs c1_mix_small_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ai}
mkdir -p $OUT
export TMPDIR=/tmp
for v in 0 1; do
  MDE_C1_MIX_SMALL=$v timeout -k 10 200 python3 -u tools/c1_accuracy_probe.py > $OUT/acc_$v.txt 2>&1
  rc=$?; echo "mix_small=$v rc=$rc"; grep -v amdgpu.ids $OUT/acc_$v.txt; [ $rc -eq 0 ] || exit $rc
done
