#!/bin/bash
# Round 6 AH: GuideDepth golden gradient-norm errors with / without the small-channel 1x1 mix kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ah}
mkdir -p $OUT
export TMPDIR=/tmp
for v in 0 1; do
  MDE_C1_MIX_SMALL=$v timeout -k 10 200 python3 -u tools/gd_grad_probe.py > $OUT/probe_$v.txt 2>&1
  rc=$?; echo "mix_small=$v rc=$rc"; grep -v amdgpu.ids $OUT/probe_$v.txt; [ $rc -eq 0 ] || exit $rc
done
