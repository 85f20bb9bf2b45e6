#!/bin/bash
# Round-5 profiles: bench lines (cfg2 fp32, cfg3 bf16, cfg4 NewCRF), kernel
# traces of the three steps, FETCH_SIZE / WRITE_SIZE passes of each
# (-> profiles/r05_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r05prof
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
}
for wl in gd_fp32 gd_bf16 nc_fp32; do
  case $wl in
    gd_fp32) args="--workload guidedepth" ;;
    gd_bf16) args="--workload guidedepth --amp bf16" ;;
    nc_fp32) args="--workload newcrf" ;;
  esac
  echo "== bench_$wl ($(date +%T))"
  timeout -k 10 400 python3 -u bench.py $args --steps 30 --warmup 5 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.log"
  rc=$?; head -c 300 "$OUT/bench_$wl.json"; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  run "trace_$wl" 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_$wl" \
      -o r05 -- python3 bench.py $args --steps 5 --warmup 3 --no-cpu-baseline
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$ctr" 400 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r05 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing
  done
done
echo done
