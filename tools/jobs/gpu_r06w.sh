#!/bin/bash
# Round 6 W: Linear weight gradients -- mde_linear_wgrad vs TunableOp's best library solution per shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06w}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/wg.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
timeout -k 10 600 python3 -u tools/lin_bench.py > $OUT/lin_tuned.log 2>&1
rc=$?; cat $OUT/lin_tuned.log | grep -v amdgpu.ids; exit $rc
