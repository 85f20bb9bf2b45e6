#!/bin/bash
# Round-4 call L: (1) bf16 3x3 conv kbench + two SQ PMC passes (verdict: what
# bounds conv3x3_fwd_bf16 / dgrad_bf16), (2) the cfg4 (newcrf) bench line and a
# rocprofv3 kernel trace of its step (window-attention backward per step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/kbench.py --only convbf > $OUT/kbench_convbf.log 2>&1
rc=$?; grep conv3x3 $OUT/kbench_convbf.log; [ $rc -eq 0 ] || exit $rc
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
  TAG=convbf1 ARGS="tools/kbench.py --only convbf --reps 10" bash tools/pmc_cmd.sh > $OUT/pmc_convbf1.txt 2>&1
rc=$?; grep -i "conv3x3_bf\|^pmc" $OUT/pmc_convbf1.txt | cut -c1-700; [ $rc -eq 0 ] || exit $rc
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
  TAG=convbf2 ARGS="tools/kbench.py --only convbf --reps 10" bash tools/pmc_cmd.sh > $OUT/pmc_convbf2.txt 2>&1
rc=$?; grep -i "conv3x3_bf\|^pmc" $OUT/pmc_convbf2.txt | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline \
  > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; python3 -c "import json;d=json.load(open('$OUT/bench_nc.json'));k=d['hip_kernels'];print(d['value'],d['ms_per_step'],{n:(k[n]['ms_per_step'],k[n].get('GBps')) for n in ('window_attn_bwd','window_attn_fwd') if n in k})"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace_nc" -o r04 \
  -- python3 bench.py --workload newcrf --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_nc.log 2>&1
rc=$?; echo "trace rc=$rc"
