#!/bin/bash
# Round-4 call Q: Winograd per-shape timing + SQ counters (what bounds the
# 16 / 32-channel variants), cfg4 bench line after the attention-bias fold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04q
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u tools/wino_bench.py > $OUT/wino.txt 2>&1
rc=$?; grep wino $OUT/wino.txt; [ $rc -eq 0 ] || exit $rc
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
  TAG=wino1 ARGS="tools/wino_bench.py --reps 5" bash tools/pmc_cmd.sh > $OUT/pmc1.txt 2>&1
rc=$?; grep -i "wino_f23\|^pmc" $OUT/pmc1.txt | cut -c1-700; [ $rc -eq 0 ] || exit $rc
PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
  TAG=wino2 ARGS="tools/wino_bench.py --reps 5" bash tools/pmc_cmd.sh > $OUT/pmc2.txt 2>&1
rc=$?; grep -i "wino_f23\|^pmc" $OUT/pmc2.txt | cut -c1-700; [ $rc -eq 0 ] || exit $rc
PMC="TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_INST_VMEM" \
  TAG=wino3 ARGS="tools/wino_bench.py --reps 5" bash tools/pmc_cmd.sh > $OUT/pmc3.txt 2>&1
rc=$?; grep -i "wino_f23\|^pmc" $OUT/pmc3.txt | cut -c1-700
timeout -k 10 600 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline \
  > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; python3 -c "import json;d=json.load(open('$OUT/bench_nc.json'));k=d['hip_kernels'];print(d['value'],d['ms_per_step'],{n:(k[n]['ms_per_step'],k[n].get('GBps')) for n in ('window_attn_bwd','window_attn_fwd') if n in k})"; exit $rc
