#!/bin/bash
# Round-3 profile set: per workload (cfg2 fp32, cfg3 bf16, cfg4 newcrf fp32):
# bench JSON line, rocprofv3 kernel-trace + stats, and separate FETCH_SIZE /
# WRITE_SIZE PMC passes -> profiles/r03_pmc_traffic_<workload>_<dtype>.json
# (tools/pmc_traffic.py, run afterwards on the CPU side).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/prof03
mkdir -p $OUT .miopen/cache .miopen/db
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=$ROOT/.miopen/cache MIOPEN_USER_DB_PATH=$ROOT/.miopen/db
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 2 "$OUT/$name.log" | cut -c1-240
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
}
for wl in ${WORKLOADS:-gd_fp32 gd_bf16 nc_fp32}; do
  case $wl in
    gd_fp32) args="--workload guidedepth" ;;
    gd_bf16) args="--workload guidedepth --amp bf16" ;;
    nc_fp32) args="--workload newcrf" ;;
  esac
  run "bench_$wl" 600 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline
  tail -n 1 "$OUT/bench_$wl.log" > "$OUT/bench_$wl.json"
  run "trace_$wl" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_$wl" \
      -o r03 -- python3 bench.py $args --steps 5 --warmup 3 --no-cpu-baseline
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$ctr" 600 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r03 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing
  done
done
echo done
