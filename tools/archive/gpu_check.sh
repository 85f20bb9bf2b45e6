#!/bin/bash
# GPU-box check: parity tests, smoke, bench.  Each GPU step has its own time
# limit; a fault/abort/timeout stops the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
# hand MIOpen's compiled kernels back (copy into .miopen/ locally) so later boxes skip the compile
# heartbeat: MIOpen's first-use kernel compiles can be silent for minutes (every step has its own timeout)
( while sleep 60; do date +%T >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB; rm -rf gpurun_out/miopen_sync && cp -r .miopen gpurun_out/miopen_sync' EXIT
STEPS=${STEPS:-10}
WARMUP=${WARMUP:-3}
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu ${TEST_TIMEOUT:-1000} python -m pytest ${TESTS:-tests} -m gpu -q -rf -x --timeout 300 -k "${PYTEST_K:-}"; rc=$?
  ok_or_testfail $rc || exit $rc
fi
if [ "${KBENCH:-1}" = 1 ]; then
  run kbench 600 python tools/kbench.py ${KB_ONLY:+--only $KB_ONLY} --json gpurun_out/kbench.json || exit $?
fi
[ "${SKIP_SMOKE:-0}" = 1 ] || run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
[ "${SKIP_BENCH:-0}" = 1 ] || run bench 900 python bench.py --steps "$STEPS" --warmup "$WARMUP" ${BENCH_ARGS:-} || exit $?
