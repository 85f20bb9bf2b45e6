#!/bin/bash
# Full -m gpu suite, then the cfg2 / cfg4 / cfg3 bench lines (no CPU baseline) on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
echo "== tests ($(date +%T))"
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 6 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "${SKIP_BENCH:-}" ] && exit 0
for tag in ${TAGS:-gd nc gd_bf16}; do
  case $tag in
    gd) a="--no-cpu-baseline";;
    gd_bf16) a="--amp bf16 --no-cpu-baseline";;
    nc) a="--workload newcrf --no-cpu-baseline";;
  esac
  timeout -k 10 300 python -u bench.py $a > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.log
  rc=$?
  echo "$tag rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/bench_$tag.json')); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
