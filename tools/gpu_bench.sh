#!/bin/bash
# bench.py lines for every workload on the box -> gpurun_out/bench_<tag>.json (+ .log).
# TAGS="gd gd_bf16 nc nc_bf16 sam" (default all); the first (gd) carries the CPU baseline.
mkdir -p gpurun_out
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db
mkdir -p "$MIOPEN_CUSTOM_CACHE_DIR" "$MIOPEN_USER_DB_PATH"
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
for tag in ${TAGS:-gd gd_bf16 nc nc_bf16 sam}; do
  case $tag in
    gd) a="";;
    gd_bf16) a="--amp bf16 --no-cpu-baseline";;
    nc) a="--workload newcrf --no-cpu-baseline";;
    nc_bf16) a="--workload newcrf --amp bf16 --no-cpu-baseline";;
    sam) a="--workload sam --no-cpu-baseline";;
    sam_bf16) a="--workload sam --amp bf16 --no-cpu-baseline";;
  esac
  timeout -k 10 420 python -u bench.py $a ${BENCH_ARGS:-} > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.log
  rc=$?
  echo "$tag rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/bench_$tag.json')); r=d['roofline'] or {}; p=d['path_roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'), 'path', p.get('frac'), 'cpu', (d['cpu_baseline'] or {}).get('value'))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
