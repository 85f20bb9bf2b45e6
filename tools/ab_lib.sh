#!/bin/bash
# Interleaved A/B of two builds of libmde_hip.so: B = $LIB_B (default the
# package's libmde_hip_ab.so), A = the in-tree library.  Runs CMD (default a
# kbench group) as A B A B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out .miopen/cache .miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db TMPDIR=/tmp
B=${LIB_B:-$PWD/monocular_depth_estimation_amd/libmde_hip_ab.so}
CMD=${CMD:-"python -u tools/kbench.py --only attn"}
for run in A B A B; do
  if [ $run = B ]; then export MDE_HIP_LIB=$B; else unset MDE_HIP_LIB; fi
  timeout -k 10 300 $CMD > gpurun_out/ablib_$run.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ablib_$run.log; exit $rc; }
  echo "== $run"; grep -v amdgpu.ids gpurun_out/ablib_$run.log | tail -n ${TAILN:-16}
done
