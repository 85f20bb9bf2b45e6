set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/.miopen/cache MIOPEN_USER_DB_PATH=$PWD/.miopen/db
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv3x3.py > gpurun_out/t_conv.log 2>&1; rc=$?
tail -15 gpurun_out/t_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --only ${KB:-conv} --json gpurun_out/kbench_conv.json > gpurun_out/kbench_conv.log 2>&1; rc=$?
cat gpurun_out/kbench_conv.log | grep -v amdgpu.ids; exit $rc
