#!/bin/bash
# Round-4 call S: Winograd (float2 staging, bank-aware pitches) tests + timing,
# cfg2 A/B of the 32-channel Winograd routing (MDE_WINO32), cfg2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_conv3x3s2.py tests/test_gpu_parity.py \
  tests/test_gpu_bf16.py -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -n 8 | cut -c1-300; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/wino_bench.py > $OUT/wino.txt 2>&1
rc=$?; grep wino $OUT/wino.txt; [ $rc -eq 0 ] || exit $rc
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_$tag.json 2> $OUT/ab_$tag.log
  local rc=$?
  echo "$tag ($*) rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$tag.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  return $rc
}
ab w64a MDE_WINO32=0 && ab w32a MDE_WINO32=1 && ab w64b MDE_WINO32=0 && ab w32b MDE_WINO32=1 || exit 1
timeout -k 10 600 python3 -u bench.py > $OUT/bench_gd.json 2> $OUT/bench_gd.log
rc=$?; echo "bench rc=$rc $(head -c 300 $OUT/bench_gd.json)"; exit $rc
