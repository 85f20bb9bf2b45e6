#!/bin/bash
# Round-5 call E: bench lines (cfg3 bf16 with convbf / with MIOpen, cfg2 fp32), 30 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp
b() {  # name env... -- args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.log
  local rc=$?
  echo "$name rc=$rc $(python3 -c "import json,sys;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
b bf16 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 || exit 1
b bf16_miopen MDE_CONVBF=0 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 || exit 1
b fp32 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 5 || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05e/bf16.json"))
ks = sorted(d["hip_kernels"].items(), key=lambda kv: -kv[1]["ms_per_step"])[:25]
for k, v in ks:
    print(f"{k:28s} {v['ms_per_step']:7.3f} ms/step  {v.get('TFLOPs', '')}")
PY
# steady-state kernel trace of the bf16 step
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gd_bf16 -- python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 8 --warmup 3 > $OUT/prof_bf16.log 2>&1 || exit 1
f=$(ls $OUT/prof/*/gd_bf16_kernel_trace.csv 2>/dev/null | head -n 1)
[ -n "$f" ] || f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_steps.py "$f" --steps 8 --top 40 > $OUT/gd_bf16_steady_state.txt && head -n 60 $OUT/gd_bf16_steady_state.txt
