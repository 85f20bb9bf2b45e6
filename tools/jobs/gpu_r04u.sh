#!/bin/bash
# Round-4 call U: wide weight-gradient block count (slab size) A/B: per-shape
# timing and PMC bytes (MDE_WIDE_BLOCKS 512 / 256), cfg2 step A/B; Winograd tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04u
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 $OUT/tests.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
for b in 512 256; do
  MDE_WIDE_BLOCKS=$b timeout -k 10 300 python3 -u tools/wred_bench.py > $OUT/wred_$b.txt 2>&1
  rc=$?; echo "WIDE_BLOCKS=$b"; grep "64->64\|128->128 s1 30\|256->256\|per cfg2" $OUT/wred_$b.txt; [ $rc -eq 0 ] || exit $rc
  for ctr in FETCH_SIZE WRITE_SIZE; do
    MDE_WIDE_BLOCKS=$b PMC=$ctr TAG=wide$b ARGS="tools/wred_bench.py" bash tools/pmc_cmd.sh > $OUT/pmc_${b}_$ctr.txt 2>&1
    grep -i "wgrad_wide_fixed_kernel<1, 80, 1, 8\|wgrad_wide_fixed_kernel<1, 40\|wgrad_wide_fixed_kernel<1, 20\|wgrad_reduce4\|^pmc" $OUT/pmc_${b}_$ctr.txt | cut -c1-250
  done
done
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_$tag.json 2> $OUT/ab_$tag.log
  local rc=$?
  echo "$tag ($*) rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$tag.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  return $rc
}
ab b512a MDE_WIDE_BLOCKS=512 && ab b256a MDE_WIDE_BLOCKS=256 && ab b512b MDE_WIDE_BLOCKS=512 && ab b256b MDE_WIDE_BLOCKS=256
