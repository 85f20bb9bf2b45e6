#!/bin/bash
# Round 6 AJ: cfg4 knob sweep on the final tree (wide wgrad blocks, Winograd minimum blocks,
# linear wgrad split target, attention backward waves a block), baseline interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06aj}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
i=0
for cfg in "" "MDE_WIDE_BLOCKS=384" "MDE_WIDE_BLOCKS=768" "" "MDE_WINO_MIN_BLOCKS=128" "MDE_WINO_MIN_BLOCKS=512" \
           "" "MDE_LIN_WGRAD_BLOCKS=384" "MDE_LIN_WGRAD_BLOCKS=768" "" ; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.log
  rc=$?; echo "[$cfg] $(python3 -c "import json;b=json.load(open('$OUT/b$i.json'));k=b['hip_kernels'];print(b['value'], *(f\"{n}={k[n]['ms_per_step']}\" for n in ('conv3x3_wgrad_wide','conv3x3_wreduce','wino_fwd','wino_dgrad','linear_wgrad','linear_wreduce') if n in k))")"; [ $rc -eq 0 ] || exit $rc
done
