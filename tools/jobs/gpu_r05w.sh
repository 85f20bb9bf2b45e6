#!/bin/bash
# Round-5 call W: conv3x3 bf16 fwd2 tile height A/B (MDE_BF_RPW) + SQ counters of the 16-channel forward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05w
mkdir -p $OUT
export TMPDIR=/tmp
for v in 1 2; do
  MDE_BF_RPW=$v timeout -k 10 200 python3 -u tools/kbench.py --only convbf > $OUT/kb_$v.log 2>&1; rc=$?; echo "rpw=$v"; grep "HIP" $OUT/kb_$v.log | grep -v wgrad; [ $rc -eq 0 ] || exit $rc
done
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" TAG=c3bf3 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|fwd2" | cut -c1-700 && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD" TAG=c3bf4 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|fwd2" | cut -c1-700
