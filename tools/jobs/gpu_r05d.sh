#!/bin/bash
# Round-5 call D: convbf parity + per-shape timing only (kernel iteration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/convbf.log 2>&1
rc=$?; echo "convbf rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/convbf.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids $OUT/kbench.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
if [ -n "${EXTRA:-}" ]; then eval "$EXTRA"; fi
