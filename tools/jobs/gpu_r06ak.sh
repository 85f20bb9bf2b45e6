#!/bin/bash
# Round 6 AK: wide weight-gradient blocks forced to 768 (MDE_WIDE_BLOCKS) vs the default rule, cfg2 and cfg4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ak}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
i=0
for wl in guidedepth newcrf; do
  for cfg in "" "MDE_WIDE_BLOCKS=768" "" "MDE_WIDE_BLOCKS=768"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python3 -u bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.log
    rc=$?; echo "$wl [$cfg] $(python3 -c "import json;b=json.load(open('$OUT/b$i.json'));k=b['hip_kernels'];print(b['value'], *(f\"{n}={k[n]['ms_per_step']}\" for n in ('conv3x3_wgrad_wide','conv3x3_wreduce') if n in k))")"; [ $rc -eq 0 ] || exit $rc
  done
done
