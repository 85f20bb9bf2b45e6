#!/bin/bash
# Quick loop: selected GPU tests (TESTS), optional kbench scripts (KB, python files), one bench (BENCH args).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
( while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ -n "${TESTS:-}" ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/q_tests.log 2>&1
  rc=$?; tail -n 4 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for kb in ${KB:-}; do
  echo "== $kb ($(date +%T))"
  timeout -k 10 300 python -u $kb > gpurun_out/q_$(basename $kb .py).log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/q_$(basename $kb .py).log | tail -n 30; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${BENCH:-}" ]; then
  echo "== bench $BENCH ($(date +%T))"
  timeout -k 10 300 python -u bench.py $BENCH --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.log
  rc=$?; python -c "
import json; d=json.load(open('gpurun_out/q_bench.json')); print(d['value'], d['ms_per_step'])
for k,v in sorted(d['hip_kernels'].items(), key=lambda kv: -kv[1]['ms_total']): print(f\"{k:26s} {v['ms_total']/3:7.3f} ms/step {v['launches']/3:5.1f}\")"; exit $rc
fi
