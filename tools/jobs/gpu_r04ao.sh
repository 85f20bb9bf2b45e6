#!/bin/bash
# Round-4 call AO: nontemporal output stores in the Winograd and direct 3x3
# conv kernels (tools/ab/libmde_hip_nt3.so): its wino / conv3x3 parity, and a
# cfg2 A/B against the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ao
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_HIP_LIB=tools/ab/libmde_hip_nt3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_conv3x3.py \
  -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests (nt3) rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
lib() { case $1 in nt3) echo tools/ab/libmde_hip_nt3.so ;; *) echo "" ;; esac; }
for v in cur nt3 cur nt3; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --steps 50 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "cfg2 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));h=d['hip_kernels'];print(d['value'], [(k, h[k]['ms_per_step']) for k in ('wino_fwd','wino_dgrad','conv3x3_fwd','conv3x3_dgrad','bn_fwd_apply','bn_fwd_stats')])")"; [ $rc -eq 0 ] || exit $rc
done
