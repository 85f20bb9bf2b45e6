#!/bin/bash
# Round 6 S: Winograd on small planes (MDE_WINO_MIN_BLOCKS) -- cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06s}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for v in 256 32 256 32 128; do
  MDE_WINO_MIN_BLOCKS=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd_b$v.json 2> $OUT/bench_gd_b$v.log
  rc=$?; echo "bench gd minblocks=$v: $(head -c 160 $OUT/bench_gd_b$v.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --workload sam --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_sam.json 2> $OUT/bench_sam.log
rc=$?; echo "bench sam: $(head -c 200 $OUT/bench_sam.json)"; exit $rc
