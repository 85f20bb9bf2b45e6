#!/bin/bash
# Round-5 call B: convbf.hip (bf16 implicit-GEMM convs) parity, per-shape
# timing vs MIOpen bf16; the data-parallel changes; the bf16 step goldens;
# cfg3 / cfg2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|no tests ran|Error|error:" $OUT/$name.log | tail -n 12 | cut -c1-300
  return $rc
}
run convbf 600 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
run kbench 300 python3 -u tools/convbf_bench.py && cat $OUT/kbench.log | cut -c1-150 || exit 1
run bn 300 python3 -u -m pytest tests/test_gpu_bn.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread
run bf16 900 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_graph_dp.py -q -rfE -p no:cacheprovider --timeout 600 --timeout-method thread || exit 1
MDE_BN_CHAN=2 run bf16_chan 600 python3 -u -m pytest tests/test_gpu_bf16.py -q -rfE -p no:cacheprovider --timeout 400 --timeout-method thread -k guidedepth -s
grep -E "HIP bf16" $OUT/bf16_chan.log | cut -c1-400
run wgrad_nc 300 python3 -u tools/wgrad_bench.py --newcrf && cat $OUT/wgrad_nc.log || exit 1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_bf16.json 2> $OUT/bench_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(head -c 300 $OUT/bench_bf16.json)"; [ $rc -eq 0 ] || exit $rc
MDE_CONVBF=0 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_bf16_miopen.json 2> $OUT/bench_bf16_miopen.log
rc=$?; echo "bench bf16 miopen rc=$rc $(head -c 300 $OUT/bench_bf16_miopen.json)"; exit $rc
