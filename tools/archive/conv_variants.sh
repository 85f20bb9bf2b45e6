#!/bin/bash
# kbench conv for each MDE_C3_VARIANT tile-shape variant (tuning experiment)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db
for v in ${VARIANTS:-0 1 2}; do
  MDE_C3_VARIANT=$v timeout -k 10 300 python tools/kbench.py --only conv --json gpurun_out/kb_conv_v$v.json \
    > gpurun_out/kb_conv_v$v.log 2>&1 || exit $?
  echo "== variant $v"; grep HIP gpurun_out/kb_conv_v$v.log
done
