#!/bin/bash
# Round-5 call U: SQ counters of the conv3x3 bf16 forward / data gradient / weight gradient (kbench convbf group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" TAG=c3bf1 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_bf" | cut -c1-600 && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" TAG=c3bf2 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_bf" | cut -c1-600
