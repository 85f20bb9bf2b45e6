#!/bin/bash
# Round 6 AN: cfg3 (bf16 autocast) knob sweep on the final tree: convbf weight-gradient blocks,
# 8-wave convbf, residual mode; baseline interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06an}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
i=0
for cfg in ${CFGS:-"" "MDE_CONVBF_WBLOCKS=512" "MDE_CONVBF_WBLOCKS=384" "" "MDE_CONVBF_NW8=1" "MDE_CONVBF_RESMODE=t21" ""}; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python3 -u bench.py --amp bf16 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.log
  rc=$?; echo "[$cfg] $(python3 -c "import json;b=json.load(open('$OUT/b$i.json'));k=b['hip_kernels'];print(b['value'], *(f\"{n}={k[n]['ms_per_step']}\" for n in k if n.startswith('convbf')))")"; [ $rc -eq 0 ] || exit $rc
done
