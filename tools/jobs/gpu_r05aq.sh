#!/bin/bash
# Round-5 call AQ: counters of the fp32 16 -> 16 full-resolution 3x3 forward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
A="tools/guide_bench.py --cin16"
timeout -k 10 200 python3 -u $A 2>&1 | grep guide && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES" TAG=c16a ARGS="$A --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-600 && \
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" TAG=c16b ARGS="$A --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-600 && \
PMC="TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_WAIT_INST_VMEM SQ_INST_CYCLES_VMEM_RD" TAG=c16c ARGS="$A --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-600
