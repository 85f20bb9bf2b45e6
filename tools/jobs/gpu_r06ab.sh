#!/bin/bash
# Round 6 AB: SQ counters of the wide 3x3 weight gradient (64->64 @60x80 bs 32, the
# cfg2 BasicBlock shape): where its 0.6 of the fp32 MFMA peak goes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ab}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 120 python3 -u tools/wgrad_bench.py --only 32,64,64,60,80 > $OUT/wb.log 2>&1
rc=$?; cat $OUT/wb.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$(pwd)/$OUT/pmc$i" -o p -- python3 tools/wgrad_bench.py --only 32,64,64,60,80 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_head.py -x -q -rfE -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_head.log 2>&1
rc=$?; echo "head tests rc=$rc"; tail -1 $OUT/tests_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nc.json 2> $OUT/bench_nc.log
rc=$?; echo "bench nc: $(python3 -c "import json;b=json.load(open('$OUT/bench_nc.json'));print(b['value'], b['hip_kernels']['head_conv_fwd'])")"; exit $rc
