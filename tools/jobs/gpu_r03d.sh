#!/bin/bash
# Round-3 call D: SSIM stream wave-order / chunk-height A/B (FETCH / WRITE
# PMC of ssim3_stream_kernel; timing in gpu_r03c.sh), then rocprofv3 kernel traces + PMC passes
# of the final tree for cfg2 (fp32) and cfg4 (newcrf) via tools/gpu_profile_r03.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ssim_ab
export TMPDIR=/tmp
for cfg in "0 5632" "1 5632" "2 5632" "2 2816"; do
  set -- $cfg
  for ctr in FETCH_SIZE WRITE_SIZE; do
    MDE_SSIM_ORDER=$1 MDE_SSIM_WAVES=$2 timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
      -d "$PWD/gpurun_out/ssim_ab/o$1_w$2_$ctr" -o p -- python3 tools/kbench.py --only loss --reps 3 \
      > gpurun_out/ssim_ab/o$1_w$2_$ctr.log 2>&1 || exit $?
  done
done
echo "ssim A/B done"
WORKLOADS="${WORKLOADS:-gd_fp32 nc_fp32}" bash tools/gpu_profile_r03.sh
