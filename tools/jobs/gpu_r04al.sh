#!/bin/bash
# Round-4 call AL: nontemporal loads / stores -- base (backward apply only,
# tools/ab/libmde_hip_base.so), bn (every BN streaming kernel,
# tools/ab/libmde_hip_bn.so), new (+ the pointwise / skip forward streams and
# the backward's gs stores, the in-tree build).  Parity of the in-tree build,
# kbench A/B, cfg2 / cfg3 bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04al
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bn.py tests/test_gpu_bf16.py tests/test_gpu_conv3x3.py -q -rfE \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
lib() { case $1 in base) echo tools/ab/libmde_hip_base.so ;; bn) echo tools/ab/libmde_hip_bn.so ;; *) echo "" ;; esac; }
for v in base bn new; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 300 python3 -u tools/kbench.py --only bn,pw > $OUT/k_$v.txt 2>&1
  rc=$?; echo "$v"; grep -E "bn\+relu|pointwise" $OUT/k_$v.txt | cut -c1-100; [ $rc -eq 0 ] || exit $rc
done
for v in base bn new base bn new; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --steps 50 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "cfg2 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));h=d['hip_kernels'];print(d['value'], [(k, h[k]['ms_per_step']) for k in ('bn_fwd_apply','bn_bwd_reduce','bn_fwd_stats','bn_bwd_apply','pointwise_fwd','pointwise_bwd','skip_reduce_fwd')])")"; [ $rc -eq 0 ] || exit $rc
done
for v in base new; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --amp bf16 --no-cpu-baseline --steps 50 > $OUT/bench_bf16_$v.json 2> $OUT/bench_bf16_$v.log
  rc=$?; echo "cfg3 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16_$v.json'));print(d['value'])")"; [ $rc -eq 0 ] || exit $rc
done
