#!/bin/bash
# Round-5 call Z: SQ / TA counters of conv3x3_bf_fwd2 (LDS-staged output) at 16 and 32 channels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" TAG=c3bf5 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|fwd2" | cut -c1-700 && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD" TAG=c3bf6 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|fwd2" | cut -c1-700 && \
PMC="TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT" TAG=c3bf7 ARGS="tools/kbench.py --only convbf --reps 5" bash tools/pmc_cmd.sh | grep -E "pmc|fwd2" | cut -c1-700
