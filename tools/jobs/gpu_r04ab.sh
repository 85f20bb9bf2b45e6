#!/bin/bash
# Round-4 call AB: refreshed PMC traffic at HEAD (FETCH_SIZE / WRITE_SIZE passes
# over cfg2 fp32, cfg3 bf16, cfg4 -> profiles/r04_pmc_traffic_*.json), the
# cfg3 bench line and kernel traces of cfg3 and cfg4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04ab
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
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$ctr" 600 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r04 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing
  done
done
run trace_gd_bf16 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_gd_bf16" \
    -o r04 -- python3 bench.py --amp bf16 --steps 5 --warmup 3 --no-cpu-baseline
run trace_nc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_nc" \
    -o r04 -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline
echo done
