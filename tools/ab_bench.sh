#!/bin/bash
# Interleaved A/B of one env switch on the cfg2 bench line: VAR=name, runs A(=1) B(=0) A B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
for v in 1 0 1 0; do
  env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-kernel-timing ${BENCH_ARGS:-} \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "$VAR=$v $(python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print(d['value'], d['ms_per_step'])")"
done
