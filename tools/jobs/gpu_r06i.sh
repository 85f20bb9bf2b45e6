#!/bin/bash
# Round 6 I: Linear weight-gradient variants (split target, prefetch distance 1 / 2), cfg4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06i}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_linear.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
MDE_LIN_WGRAD_PD=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_linear.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests32.log 2>&1
rc=$?; echo "tests pd1 rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests32.log | tail -5 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for cfg in "2 1024" "2 512" "2 768" "1 512"; do
  set -- $cfg
  MDE_LIN_WGRAD_PD=$1 MDE_LIN_WGRAD_BLOCKS=$2 timeout -k 10 300 python3 -u tools/lin_bench.py > $OUT/lin_$1_$2.log 2>&1
  rc=$?; echo "pd=$1 blocks=$2"; grep -E "T=( 76800|307200)|total" $OUT/lin_$1_$2.log | sed 's/hipBLASLt.*hip /hip /'; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc: $(head -c 200 $OUT/bench_nc.json)"; exit $rc
