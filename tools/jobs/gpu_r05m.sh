#!/bin/bash
# Round-5 call M: convbf weight-gradient occupancy / grid A/B + parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/convbf.log 2>&1
rc=$?; echo "convbf rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/convbf.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for b in 256 512; do
  MDE_CONVBF_WBLOCKS=$b timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench_$b.log 2>&1
  rc=$?; echo "kbench WBLOCKS=$b rc=$rc"; grep -v amdgpu.ids $OUT/kbench_$b.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
