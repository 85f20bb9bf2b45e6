#!/bin/bash
# Round-5 call AE: SQ counters of the Winograd kernels (tools/wino_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/wino_bench.py 2>&1 | grep -v amdgpu.ids | tail -8
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" TAG=wino5a ARGS="tools/wino_bench.py" bash tools/pmc_cmd.sh | grep -E "pmc|wino_f23" | cut -c1-600 && \
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" TAG=wino5b ARGS="tools/wino_bench.py" bash tools/pmc_cmd.sh | grep -E "pmc|wino_f23" | cut -c1-600 && \
PMC="TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_INST_VMEM" TAG=wino5c ARGS="tools/wino_bench.py" bash tools/pmc_cmd.sh | grep -E "pmc|wino_f23" | cut -c1-600
