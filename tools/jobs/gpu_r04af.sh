#!/bin/bash
# Round-4 call AF: which ATen ops launch the remaining elementwise kernels of a
# cfg2 step (fp32) and of a cfg3 step (bf16 autocast).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04af
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --top 30 > $OUT/aten_fp32.txt 2>&1
rc=$?; echo "fp32 rc=$rc"; tail -n 32 $OUT/aten_fp32.txt | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --top 30 --amp bf16 > $OUT/aten_bf16.txt 2>&1
rc=$?; echo "bf16 rc=$rc"; tail -n 32 $OUT/aten_bf16.txt | cut -c1-200
