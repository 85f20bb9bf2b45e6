#!/bin/bash
# Round-4 call K: cfg2 A/B of the small-tensor BN kernels (MDE_BN_CHAN) with the
# small-launch sum from the bench's per-kernel times, the cfg2 bench line, the
# cfg3 GUIDE_BF16 A/B, a rocprofv3 kernel trace of the cfg2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04k
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
SUM="import json,sys;d=json.load(open(sys.argv[1]));k=d['hip_kernels'];ns=('bn_fwd_final','bn_fwd_apply_small','bn_bwd_apply_small','conv3x3_wreduce','se_bwd_fc');print(d['value'],d['ms_per_step'],'small-launch ms/step',round(sum(k.get(n,{}).get('ms_per_step',0) for n in ns),3),{n:k.get(n,{}).get('ms_per_step') for n in ns+('ssim3_l1','bn_fwd_stats','bn_bwd_reduce')})"
for v in 0 1; do
  MDE_BN_CHAN=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline \
    > $OUT/ab_chan_$v.json 2> $OUT/ab_chan_$v.log
  rc=$?; echo "BN_CHAN=$v rc=$rc $(python3 -c "$SUM" $OUT/ab_chan_$v.json 2>&1)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 -u bench.py > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench rc=$rc $(python3 -c "$SUM" $OUT/bench_gd.json 2>&1)"; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MDE_GUIDE_BF16=$v timeout -k 10 300 python3 -u bench.py --amp bf16 --steps 30 --warmup 10 --no-cpu-baseline \
    --no-kernel-timing > $OUT/ab_bf16_$v.json 2> $OUT/ab_bf16_$v.log
  rc=$?; echo "GUIDE_BF16=$v rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_bf16_$v.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd" -o r04 \
  -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_gd.log 2>&1
rc=$?; echo "trace rc=$rc"
