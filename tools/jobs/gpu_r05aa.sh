#!/bin/bash
# Round-5 call AA: texture-addresser / SQ load of the convbf kernels (convbf_bench, all cfg3 shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC="TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" TAG=cbfta ARGS="tools/convbf_bench.py" bash tools/pmc_cmd.sh | grep -E "pmc|convbf_(fwd|wgrad)" | cut -c1-600
