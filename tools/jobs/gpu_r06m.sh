#!/bin/bash
# Round 6 M: cfg4 op attribution after the 1x1 / wgrad work; cfg2 C1_PAD sanity A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06m}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload newcrf --bs 16 --top 30 > $OUT/aten_nc.log 2>&1
rc=$?; echo "aten nc rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_C1_PAD=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd_c$v.json 2> $OUT/bench_gd_c$v.log
  rc=$?; echo "bench gd c1pad=$v: $(head -c 160 $OUT/bench_gd_c$v.json)"; [ $rc -eq 0 ] || exit $rc
done
