#!/bin/bash
# Round-4 call V: bf16 3x3 conv tile height A/B (MDE_BF_RPW 1 / 2): parity
# tests with 8-row tiles, kbench per pass, cfg3 step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04v
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MDE_BF_RPW=2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_conv3x3.py -q -rfE \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests (RPW=2) rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -n 6 | cut -c1-300; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  MDE_BF_RPW=$r timeout -k 10 300 python3 -u tools/kbench.py --only convbf > $OUT/convbf_$r.txt 2>&1
  rc=$?; echo "RPW=$r"; grep "HIP" $OUT/convbf_$r.txt | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --amp bf16 --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_$tag.json 2> $OUT/ab_$tag.log
  local rc=$?
  echo "$tag ($*) rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$tag.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  return $rc
}
ab r1a MDE_BF_RPW=1 && ab r2a MDE_BF_RPW=2 && ab r1b MDE_BF_RPW=1 && ab r2b MDE_BF_RPW=2
