#!/bin/bash
# Round-5 call R: decoder 32 -> 32 3x3 convs: conv3x3 bf16 kernel vs convbf (kernels, cfg3 step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/convbf_bench.py --only 32,32,240,320,3,1 > $OUT/cbf32.log 2>&1; rc=$?; cat $OUT/cbf32.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/convbf_bench.py --only 64,64,120,160,3,1 > $OUT/cbf64.log 2>&1; rc=$?; grep "(64" $OUT/cbf64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/kbench.py --only convbf > $OUT/kb.log 2>&1; rc=$?; grep conv3x3 $OUT/kb.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_C3BF32=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  rc=$?; echo "c3bf32=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if 'conv' in n])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
