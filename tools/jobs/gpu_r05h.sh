#!/bin/bash
# Round-5 call H: convbf parity under each resident-filter variant, then the
# per-shape timing of each (MDE_CONVBF_RESMODE = t22 / t21).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
for m in t22 t21; do
  MDE_CONVBF_RESMODE=$m timeout -k 10 300 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/convbf_$m.log 2>&1
  rc=$?; echo "convbf $m rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/convbf_$m.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
done
for m in t22 t21; do
  MDE_CONVBF_RESMODE=$m timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench_$m.log 2>&1
  rc=$?; echo "kbench $m rc=$rc"; grep -v amdgpu.ids $OUT/kbench_$m.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
