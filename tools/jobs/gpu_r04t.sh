#!/bin/bash
# Round-4 call T: FETCH_SIZE / WRITE_SIZE PMC passes over the cfg2 fp32, cfg3
# bf16 and cfg4 steps (-> profiles/r04_pmc_traffic_<workload>_<dtype>.json via
# tools/pmc_traffic.py on the CPU side), the cfg3 bench line + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04t
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
run bench_gd_bf16 600 python3 bench.py --amp bf16 --steps 50 --warmup 10 --no-cpu-baseline
tail -n 1 "$OUT/bench_gd_bf16.log" > "$OUT/bench_gd_bf16.json"
run trace_gd_bf16 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd_bf16" \
    -o r04 -- python3 bench.py --amp bf16 --steps 5 --warmup 3 --no-cpu-baseline
for wl in gd_fp32 gd_bf16 nc_fp32; do
  case $wl in
    gd_fp32) args="--workload guidedepth" ;;
    gd_bf16) args="--workload guidedepth --amp bf16" ;;
    nc_fp32) args="--workload newcrf" ;;
  esac
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$ctr" 600 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r04 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing
  done
done
echo done
