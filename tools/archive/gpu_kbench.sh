#!/bin/bash
# kernel micro-benchmarks (+ optional parity subset) on the box.
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread > gpurun_out/ktests.log 2>&1
  rc=$?; tail -n 3 gpurun_out/ktests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u tools/kbench.py --only ${ONLY:-resize,dw} --json gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1
rc=$?; cat gpurun_out/kbench.log | grep -v amdgpu.ids; exit $rc
