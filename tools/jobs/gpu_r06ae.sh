#!/bin/bash
# Round 6 AE: fp32 x2 resizes -- flat two-column forward (MDE_X2_FWD) and 16-row bands (MDE_X2_ROWS):
# resize parity tests, kbench per variant, cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ae}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for cfg in "0 8" "1 8" "0 16" "1 16"; do
  set -- $cfg
  MDE_X2_FWD=$1 MDE_X2_ROWS=$2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_se_bn.py -k "bilinear or resize or grad_slot" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_f$1_r$2.log 2>&1
  rc=$?; echo "tests fwd=$1 rows=$2 rc=$rc $(tail -1 $OUT/tests_f$1_r$2.log)"; [ $rc -eq 0 ] || exit $rc
  MDE_X2_FWD=$1 MDE_X2_ROWS=$2 timeout -k 10 200 python3 -u tools/kbench.py --only resize > $OUT/kb_f$1_r$2.txt 2>&1
  rc=$?; echo "kbench fwd=$1 rows=$2 rc=$rc"; grep "x2" $OUT/kb_f$1_r$2.txt | grep -v bf16; [ $rc -eq 0 ] || exit $rc
done
for cfg in "0 8" "1 16" "0 8" "1 16"; do
  set -- $cfg
  MDE_X2_FWD=$1 MDE_X2_ROWS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_gd_f$1_r$2.json 2> $OUT/bench_gd_f$1_r$2.log
  rc=$?; echo "bench gd fwd=$1 rows=$2: $(python3 -c "import json;b=json.load(open('$OUT/bench_gd_f$1_r$2.json'));k=b['hip_kernels'];print(b['value'], k['bilinear_fwd']['ms_per_step'], k['bilinear_bwd']['ms_per_step'], b['path_roofline']['frac'])")"; [ $rc -eq 0 ] || exit $rc
done
