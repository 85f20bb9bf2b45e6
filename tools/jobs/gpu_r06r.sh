#!/bin/bash
# Round 6 R: cfg2 after the biased-1x1 route: attribution + A/B (MDE_CHANSUM gates the biased 1x1 / bias-gradient routes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06r}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/aten_ops_profile.py --workload guidedepth --bs 32 --top 40 > $OUT/aten_gd.log 2>&1
rc=$?; echo "aten gd rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MDE_CHANSUM=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_gd_s$v.json 2> $OUT/bench_gd_s$v.log
  rc=$?; echo "bench gd chansum=$v: $(head -c 160 $OUT/bench_gd_s$v.json)"; [ $rc -eq 0 ] || exit $rc
done
