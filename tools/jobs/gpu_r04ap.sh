#!/bin/bash
# Round-4 call AP: __graft_entry__.smoke() on the final tree (as the driver runs it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04ap
timeout -k 10 600 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04ap/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 5 gpurun_out/r04ap/smoke.log | cut -c1-300
