#!/bin/bash
# Round-5 call AL: the guide convs (3 input channels): timing and SQ / TA counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/guide_bench.py 2>&1 | grep guide && \
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" TAG=guide_a ARGS="tools/guide_bench.py --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-700 && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAVES" TAG=guide_b ARGS="tools/guide_bench.py --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-700 && \
PMC="TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_WAIT_INST_VMEM SQ_INST_CYCLES_VMEM_RD" TAG=guide_c ARGS="tools/guide_bench.py --reps 3" bash tools/pmc_cmd.sh | grep -E "pmc|conv3x3_fwd" | cut -c1-700
