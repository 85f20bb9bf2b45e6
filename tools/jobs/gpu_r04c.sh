#!/bin/bash
# Round-4 call C: per-shape vendor kernels of the convolutions still on MIOpen
# (tools/conv_kernel_map.py), then the cfg2 bench with MIOpen's NHWC implicit
# GEMM solvers switched off (MIOpen then picks NCHW solvers: no transposes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/conv_kernel_map.py > $OUT/conv_map.txt 2>&1
rc=$?; echo "conv_map rc=$rc"; [ $rc -eq 0 ] || exit $rc
NHWC0="MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0"
env $NHWC0 timeout -k 10 300 python3 -u tools/conv_kernel_map.py > $OUT/conv_map_nonhwc.txt 2>&1
rc=$?; echo "conv_map nonhwc rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in base nonhwc base nonhwc; do
  if [ $v = base ]; then e="A=1"; else e="$NHWC0"; fi
  env $e timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_$v.json 2> $OUT/ab_$v.log
  rc=$?; echo "$v rc=$rc $(head -c 160 $OUT/ab_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
# wide weight gradient: XCD-aware tile walk (A = in-tree) vs round-3 walk (B = libmde_hip_ab.so)
CMD="python3 -u tools/wgrad_bench.py" TAILN=14 bash tools/ab_lib.sh
rc=$?; echo "ab_lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
PMC=FETCH_SIZE TAG=wgA ARGS="tools/wgrad_bench.py" bash tools/pmc_cmd.sh | grep -i "wgrad\|pmc" || exit 1
MDE_HIP_LIB=$PWD/monocular_depth_estimation_amd/libmde_hip_ab.so PMC=FETCH_SIZE TAG=wgB ARGS="tools/wgrad_bench.py" \
  bash tools/pmc_cmd.sh | grep -i "wgrad\|pmc" || exit 1
