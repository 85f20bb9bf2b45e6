#!/bin/bash
# Round-3 call A: new / changed GPU tests, Depth_Loss kbench, PMC width
# calibration, the full suite, the bench, MIOpen weight-gradient solver A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/calib .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
step() { echo "== $1 ($(date +%T))"; }
step "new tests"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_graph.py::test_bucketed_overlapped_allreduce_graph_matches_eager" \
  tests/test_gpu_graph_dp.py tests/test_gpu_resume.py \
  "tests/test_gpu_parity.py::test_guided_block_variants_golden" \
  "tests/test_gpu_parity.py::test_guidedepth_s_golden" \
  tests/test_gpu_parity.py -k "depth_loss or variants or guidedepth_s or bucketed or graph_trainer or resume" \
  > gpurun_out/new_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/new_tests.log; [ $rc -le 1 ] || exit $rc
step "kbench loss"
timeout -k 10 300 python -u tools/kbench.py --only loss > gpurun_out/kbench_loss.log 2>&1
rc=$?; cat gpurun_out/kbench_loss.log | tail -n 8; [ $rc -eq 0 ] || exit $rc
step "calib"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/calib/$ctr" -o calib \
    -- ./tools/calib/pmc_calib > gpurun_out/calib/$ctr.log 2>&1
  rc=$?; echo "calib $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
step "full suite"
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 8 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
step "bench"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_gd.json 2> gpurun_out/bench_gd.log
rc=$?; tail -c 400 gpurun_out/bench_gd.json; [ $rc -eq 0 ] || exit $rc
for v in nowrwnhwc nonhwc; do
  step "ab $v"
  case $v in
    nowrwnhwc) e="MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0";;
    nonhwc) e="MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0";;
  esac
  env $e timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log
  rc=$?; echo "$v rc=$rc $(head -c 200 gpurun_out/ab_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
