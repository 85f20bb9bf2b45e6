#!/bin/bash
# Round-6 profiles: per workload
# the FETCH_SIZE / WRITE_SIZE passes FIRST, reduced to
# profiles/r06_pmc_traffic_<tag>.json on the box so the bench line that
# follows prices its roofline traffic from this tree's counters; then the
# kernel trace and the bench line.  Args: workloads (gd_fp32 gd_bf16 nc_fp32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=gpurun_out/${TAGDIR:-r06prof}
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
for wl in "$@"; do
  case $wl in
    gd_fp32) args="--workload guidedepth"; tag=guidedepth_fp32 ;;
    gd_bf16) args="--workload guidedepth --amp bf16"; tag=guidedepth_bf16 ;;
    nc_fp32) args="--workload newcrf"; tag=newcrf_fp32 ;;
  esac
  # the profiled runs keep MIOpen's user db / kernel cache to themselves: a
  # bench line after them on the same box ran 938 instead of 971-976 img/s
  # with different MIOpen solvers (${TAGDIR:-r06prof}, first attempt)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    MIOPEN_USER_DB_PATH=/tmp/mio_prof/db MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_prof/cache \
    run "pmc_${wl}_$ctr" 400 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$OUT/pmc_${wl}_$ctr" \
        -o r06 -- python3 bench.py $args --steps 2 --warmup 2 --no-cpu-baseline --no-kernel-timing
  done
  python3 tools/pmc_traffic.py "$OUT/pmc_${wl}_FETCH_SIZE/r06_counter_collection.csv" \
      "$OUT/pmc_${wl}_WRITE_SIZE/r06_counter_collection.csv" -o "profiles/r06_pmc_traffic_$tag.json" > /dev/null || exit 1
  cp "profiles/r06_pmc_traffic_$tag.json" "$OUT/"
  rm -rf "$OUT/pmc_${wl}_FETCH_SIZE" "$OUT/pmc_${wl}_WRITE_SIZE"
  MIOPEN_USER_DB_PATH=/tmp/mio_trace_$wl/db MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_trace_$wl/cache \
  run "trace_$wl" 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_$wl" \
      -o r06 -- python3 bench.py $args --steps 5 --warmup 3 --no-cpu-baseline
  echo "== bench_$wl ($(date +%T))"
  timeout -k 10 400 python3 -u bench.py $args --steps 30 --warmup 5 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.log"
  rc=$?; head -c 300 "$OUT/bench_$wl.json"; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
done
echo done
