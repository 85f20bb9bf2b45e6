#!/bin/bash
# Round 6 U: the vendor GEMM solution table -- TunableOp tuning over the bench
# workloads (cfg4, SAM, cfg2, cfg3), one file; then A/B with the table loaded
# read-only by gemm_table.enable() vs MDE_GEMM_TABLE=0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06u}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for wl in "--workload newcrf" "--workload sam" "--workload guidedepth --amp bf16"; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/table.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 timeout -k 10 400 python3 -u bench.py $wl --steps 3 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/tune.json 2> $OUT/tune.log
  rc=$?; echo "tune [$wl] rc=$rc $(wc -l < $OUT/table0.csv) lines"; [ $rc -eq 0 ] || exit $rc
done
cp $OUT/table0.csv monocular_depth_estimation_amd/tunableop_gfx950.csv
for v in 0 1; do
  for wl in newcrf sam; do
    MDE_GEMM_TABLE=$v timeout -k 10 300 python3 -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_${wl}_t$v.json 2> $OUT/bench_${wl}_t$v.log
    rc=$?; echo "bench $wl table=$v: $(head -c 150 $OUT/bench_${wl}_t$v.json | cut -c100-150) $(grep -o '"gemm_table": [^,]*' $OUT/bench_${wl}_t$v.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
