#!/bin/bash
# Round 6 AL: wide weight-gradient blocks -- 768 for >= 64 channel groups (new default) vs 256
# forced (the old rule's value at those shapes): conv3x3 / NewCRF tests, cfg4 and cfg2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06al}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_newcrf.py tests/test_gpu_wino.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -eq 0 ] || exit $rc
i=0
for wl in newcrf guidedepth; do
  for cfg in "MDE_WIDE_BLOCKS=256" "" "MDE_WIDE_BLOCKS=256" ""; do
    [ $wl = guidedepth ] && [ -n "$cfg" ] && continue
    i=$((i+1))
    env $cfg timeout -k 10 300 python3 -u bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.log
    rc=$?; echo "$wl [$cfg] $(python3 -c "import json;b=json.load(open('$OUT/b$i.json'));k=b['hip_kernels'];print(b['value'], *(f\"{n}={k[n]['ms_per_step']}\" for n in ('conv3x3_wgrad_wide','conv3x3_wreduce') if n in k))")"; [ $rc -eq 0 ] || exit $rc
  done
done
