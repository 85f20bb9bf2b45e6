#!/bin/bash
# Round-4 call AM: parity of the in-tree build (nontemporal hints as kept), and
# an A/B against tools/ab/libmde_hip_nt2.so (+ nontemporal stores in the x2
# resizes and the SE streams): cfg2 interleaved, cfg3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04am
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_bn.py tests/test_gpu_bf16.py tests/test_gpu_conv3x3.py tests/test_gpu_parity.py \
  tests/test_gpu_se_bn.py -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
lib() { case $1 in nt2) echo tools/ab/libmde_hip_nt2.so ;; *) echo "" ;; esac; }
for v in cur nt2 cur nt2; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --steps 50 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "cfg2 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));h=d['hip_kernels'];print(d['value'], [(k, h[k]['ms_per_step']) for k in ('bilinear_fwd','bilinear_bwd','se_scale','se_bwd_apply','se_squeeze','bn_bwd_apply')])")"; [ $rc -eq 0 ] || exit $rc
done
for v in cur nt2; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --amp bf16 --no-cpu-baseline --steps 50 > $OUT/bench_bf16_$v.json 2> $OUT/bench_bf16_$v.log
  rc=$?; echo "cfg3 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16_$v.json'));print(d['value'], d['path_roofline']['frac'])")"; [ $rc -eq 0 ] || exit $rc
done
