#!/bin/bash
# Round-3 call C: full -m gpu suite, bench lines (cfg2 fp32, cfg4, cfg3 bf16),
# ATen-op attribution of the cfg2 step, SSIM stream chunk-height A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests"
PYTEST_ARGS="-rxX" bash tools/gpu_tests.sh
trc=$?
[ $trc -le 1 ] || exit $trc
step "bench"
TAGS="gd nc gd_bf16" bash tools/gpu_bench.sh || exit $?
step "aten ops"
timeout -k 10 300 python -u tools/aten_ops_profile.py > gpurun_out/aten_ops.txt 2>&1 || exit $?
step "ssim chunk A/B"
for rep in 1 2; do
  for cfg in "0 5632" "1 5632" "2 5632" "0 2816" "1 2816" "2 2816"; do
    set -- $cfg
    echo "order=$1 waves=$2 rep=$rep: $(MDE_SSIM_ORDER=$1 MDE_SSIM_WAVES=$2 timeout -k 10 120 python -u tools/kbench.py --only loss 2>&1 | grep ssim3)"
  done
done
exit $trc
