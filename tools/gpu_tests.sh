#!/bin/bash
# Full -m gpu suite on the box (one process, per-test timeout), log under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -n 5 gpurun_out/gpu_tests.log
exit $rc
