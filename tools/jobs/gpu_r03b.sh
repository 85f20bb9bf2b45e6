#!/bin/bash
# Round-3 call B: window-attention backward at three waves per SIMD, packed
# Depth_Loss, bf16 MFMA conv3x3 -- tests, kbench, cfg4 + cfg3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
step() { echo "== $1 ($(date +%T))"; }
step "conv tests"
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_conv3x3.py tests/test_gpu_bn.py > gpurun_out/b_conv.log 2>&1
rc=$?; tail -n 6 gpurun_out/b_conv.log; [ $rc -le 1 ] || exit $rc
step "tests"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_newcrf.py tests/test_gpu_sam.py tests/test_gpu_resume.py tests/test_gpu_bf16.py \
  "tests/test_gpu_parity.py::test_depth_loss_golden" "tests/test_gpu_parity.py::test_depth_loss_streaming_shapes_vs_oracle" "tests/test_gpu_parity.py::test_depth_loss_full_size_vs_oracle_crop" \
  > gpurun_out/b_tests.log 2>&1
rc=$?; tail -n 8 gpurun_out/b_tests.log; [ $rc -le 1 ] || exit $rc
step "kbench"
timeout -k 10 300 python -u tools/kbench.py --only attn,loss > gpurun_out/kbench_attn.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kbench_attn.log | tail -n 16; [ $rc -eq 0 ] || exit $rc
step "bench newcrf"
timeout -k 10 600 python -u bench.py --workload newcrf --no-cpu-baseline > gpurun_out/bench_nc.json 2> gpurun_out/bench_nc.log
rc=$?; python -c "
import json; d=json.load(open('gpurun_out/bench_nc.json')); print(d['value'], d['ms_per_step'])
for k in ('window_attn_bwd','window_attn_fwd'): print(k, d['hip_kernels'].get(k))"; [ $rc -eq 0 ] || exit $rc
step "bench gd bf16"
timeout -k 10 600 python -u bench.py --amp bf16 --no-cpu-baseline > gpurun_out/bench_gd_bf16.json 2> gpurun_out/bench_gd_bf16.log
rc=$?; python -c "
import json; d=json.load(open('gpurun_out/bench_gd_bf16.json')); print(d['value'], d['ms_per_step'])
for k in ('conv3x3_fwd','conv3x3_dgrad','conv3x3_wgrad'): print(k, d['hip_kernels'].get(k))"; exit $rc
