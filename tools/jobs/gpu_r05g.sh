#!/bin/bash
# Round-5 call G: convbf parity + per-shape timing, A/B of the 64 x 64 wave
# tiles (MDE_CONVBF_T22=0 -> 32 x 64), then the SQ counters (gpu_r05c.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/convbf.log 2>&1
rc=$?; echo "convbf rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/convbf.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids $OUT/kbench.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
MDE_CONVBF_T22=0 timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench_t21.log 2>&1
rc=$?; echo "kbench T22=0 rc=$rc"; grep -v amdgpu.ids $OUT/kbench_t21.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r05c.sh
