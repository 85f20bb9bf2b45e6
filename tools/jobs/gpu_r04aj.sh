#!/bin/bash
# Round-4 call AJ / AN: final refresh at HEAD -- full GPU suite, the cfg2 / cfg3 /
# cfg4 bench lines (with the CPU baseline), a cfg2 kernel trace, and the PMC
# traffic passes of all three workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04an
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
AMD_LOG_LEVEL=1 timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -v "Cannot find the function" $OUT/suite.log | grep -E "^FAILED|^ERROR|passed|failed" | tail -n 12 | cut -c1-300
[ $rc -le 1 ] || exit $rc
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.log"
  local rc=$?
  echo "$name rc=$rc $(head -c 160 $OUT/$name.out)"
  [ $rc -eq 0 ] || exit $rc
}
run bench_gd 600 python3 -u bench.py
run bench_gd_bf16 600 python3 -u bench.py --amp bf16
run bench_nc 600 python3 -u bench.py --workload newcrf
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd" -o r04 \
  -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_gd.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for wl in gd_fp32 gd_bf16 nc_fp32; do
  case $wl in
    gd_fp32) args="--workload guidedepth" ;;
    gd_bf16) args="--workload guidedepth --amp bf16" ;;
    nc_fp32) args="--workload newcrf" ;;
  esac
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r04 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing \
        > "$OUT/pmc_${wl}_$ctr.log" 2>&1
    rc=$?; echo "pmc $wl $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo done
