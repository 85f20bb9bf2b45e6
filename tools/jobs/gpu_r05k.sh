#!/bin/bash
# Round-5 call K: bf16 pointwise backward prefetch kernel A/B + bf16 tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bf16.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread -k "pointwise or bn_relu or pw" > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|deselected" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/pw_bf16_bench.py > $OUT/pw.log 2>&1; rc=$?; grep -v amdgpu $OUT/pw.log; [ $rc -eq 0 ] || exit $rc
MDE_PW_PF=0 timeout -k 10 120 python3 -u tools/pw_bf16_bench.py > $OUT/pw0.log 2>&1; rc=$?; grep -v amdgpu $OUT/pw0.log; exit $rc
