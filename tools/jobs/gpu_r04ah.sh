#!/bin/bash
# Round-4 call AH: pointwise forward with the next tile's operands prefetched
# (narrow inputs): parity (skip / pointwise / bf16), kbench pw A/B against the
# previous build (tools/ab/libmde_hip_base.so), cfg2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ah
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_conv3x3.py tests/test_gpu_se_bn.py -q -rfE \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|no tests ran|not found" $OUT/tests.log | tail -n 8 | cut -c1-300; [ $rc -le 1 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then L=tools/ab/libmde_hip_base.so; else L=; fi
  MDE_HIP_LIB=$L timeout -k 10 300 python3 -u tools/kbench.py --only pw > $OUT/pw_$v.txt 2>&1
  rc=$?; echo "$v"; grep pointwise $OUT/pw_$v.txt | cut -c1-100; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench gd rc=$rc $(head -c 200 $OUT/bench_gd.json)"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench_gd.json'));print({k:v for k,v in d['hip_kernels'].items() if 'pointwise' in k})"
