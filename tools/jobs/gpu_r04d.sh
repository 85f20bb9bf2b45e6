#!/bin/bash
# Round-4 call D: (1) the full GPU suite with the overlapped scheme as the
# N > 1 default and no xfail (HIP error log on, so an abort of the RCCL child
# shows its message in the failure), (2) bf16 3x3 conv kbench + two SQ PMC
# passes, (3) cfg4 (newcrf) bench line + rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04d
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 TMPDIR=/tmp
AMD_LOG_LEVEL=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rfE -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -v "Cannot find the function" $OUT/suite.log | tail -n 25 | cut -c1-400
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/kbench.py --only convbf > $OUT/kbench_convbf.log 2>&1
rc=$?; grep conv3x3 $OUT/kbench_convbf.log; [ $rc -eq 0 ] || exit $rc
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
  TAG=convbf1 ARGS="tools/kbench.py --only convbf --reps 10" bash tools/pmc_cmd.sh | grep -i "conv3x3_bf\|pmc" | cut -c1-600
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
  TAG=convbf2 ARGS="tools/kbench.py --only convbf --reps 10" bash tools/pmc_cmd.sh | grep -i "conv3x3_bf\|pmc" | cut -c1-600
timeout -k 10 600 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline \
  > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; head -c 300 $OUT/bench_nc.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_nc" -o r04 \
  -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace rc=$rc"
