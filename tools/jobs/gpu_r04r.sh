#!/bin/bash
# Round-4 call R: Winograd with coalesced float2 input staging: tests, per-shape
# timing, SQ / TA counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04r
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/tests.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/wino_bench.py > $OUT/wino.txt 2>&1
rc=$?; grep wino $OUT/wino.txt; [ $rc -eq 0 ] || exit $rc
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
  TAG=winob1 ARGS="tools/wino_bench.py --reps 5" bash tools/pmc_cmd.sh > $OUT/pmc1.txt 2>&1
rc=$?; grep -i "wino_f23\|^pmc" $OUT/pmc1.txt | cut -c1-700; [ $rc -eq 0 ] || exit $rc
PMC="TA_BUSY_avr SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  TAG=winob2 ARGS="tools/wino_bench.py --reps 5" bash tools/pmc_cmd.sh > $OUT/pmc2.txt 2>&1
rc=$?; grep -i "wino_f23\|^pmc" $OUT/pmc2.txt | cut -c1-700
