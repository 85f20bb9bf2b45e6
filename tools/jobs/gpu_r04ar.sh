#!/bin/bash
# Round-4 call AR: nontemporal gq / gk / gv stores in the window-attention
# backward (tools/ab/libmde_hip_nt4.so): NewCRF / SAM parity with that build,
# cfg4 A/B against the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ar
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_HIP_LIB=tools/ab/libmde_hip_nt4.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_newcrf.py tests/test_gpu_sam.py \
  -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests (nt4) rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
lib() { case $1 in nt4) echo tools/ab/libmde_hip_nt4.so ;; *) echo "" ;; esac; }
for v in cur nt4 cur nt4; do
  MDE_HIP_LIB=$(lib $v) timeout -k 10 600 python3 -u bench.py --workload newcrf --no-cpu-baseline --steps 40 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "cfg4 $v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));r=d['roofline'];print(d['value'], r['kernel'], r['ms_per_step'], r['frac'])")"; [ $rc -eq 0 ] || exit $rc
done
