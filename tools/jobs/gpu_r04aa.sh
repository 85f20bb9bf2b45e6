#!/bin/bash
# Round-4 call AA: SSIM pair kernel with corrected-reciprocal divisions, SGPR
# row offsets, 3 waves / SIMD; attention slab reduce under its own timing id.
# Parity (ssim / loss / attention), kbench loss, cfg2 + cfg4 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04aa
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_newcrf.py -q -rfE -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 12 | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/kbench.py --only loss > $OUT/kbench_loss.txt 2>&1
rc=$?; grep -v "^\s*$" $OUT/kbench_loss.txt | tail -n 6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 200 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd.json'));print(d['hip_kernels'].get('ssim3_l1'))"
timeout -k 10 600 python3 -u bench.py --workload newcrf --no-cpu-baseline > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc rc=$rc $(head -c 200 $OUT/bench_nc.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_nc.json'));print(d['roofline']);print(d['hip_kernels'].get('window_attn_bwd_reduce'))"
