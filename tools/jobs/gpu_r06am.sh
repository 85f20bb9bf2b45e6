#!/bin/bash
# Round 6 AM: cfg2 wide weight-gradient block count sweep (MDE_WIDE_BLOCKS forced for every shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06am}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
i=0
for cfg in "" "MDE_WIDE_BLOCKS=384" "MDE_WIDE_BLOCKS=512" "" "MDE_WIDE_BLOCKS=384" "MDE_WIDE_BLOCKS=512" "MDE_WIDE_BLOCKS=192"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.log
  rc=$?; echo "[$cfg] $(python3 -c "import json;b=json.load(open('$OUT/b$i.json'));k=b['hip_kernels'];print(b['value'], *(f\"{n}={k[n]['ms_per_step']}\" for n in ('conv3x3_wgrad_wide','conv3x3_wreduce') if n in k))")"; [ $rc -eq 0 ] || exit $rc
done
