#!/bin/bash
# A/B of MIOpen solver choices for the cfg2 step (env switches of MIOpen's own
# solver list); each variant is one bench run, results in gpurun_out/ab_*.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
( while sleep 60; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
run() {
  local tag=$1; shift
  echo "== $tag ($(date +%T))"
  env "$@" timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "gpurun_out/ab_$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc"; tail -n 1 "gpurun_out/ab_$tag.log" | cut -c1-200
  return $rc
}
run base A=1 || exit $?
run nowrwnhwc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 || exit $?
run nonhwc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 \
  MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 \
  MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 || exit $?
