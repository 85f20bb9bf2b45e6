#!/bin/bash
# Round-4 call AK: BN backward apply with nontemporal loads / stores: BN
# parity, kbench bn A/B against the previous build, cfg2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ak
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bn.py -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then L=tools/ab/libmde_hip_base.so; else L=; fi
  MDE_HIP_LIB=$L timeout -k 10 300 python3 -u tools/kbench.py --only bn > $OUT/bn_$v.txt 2>&1
  rc=$?; echo "$v"; grep "bwd" $OUT/bn_$v.txt | grep -v MIOpen | cut -c1-100; [ $rc -eq 0 ] || exit $rc
done
for v in base new; do
  if [ $v = base ]; then L=tools/ab/libmde_hip_base.so; else L=; fi
  MDE_HIP_LIB=$L timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "bench $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'], d['roofline']['frac'], d['hip_kernels']['bn_bwd_apply'])")"; [ $rc -eq 0 ] || exit $rc
done
