#!/bin/bash
# Round-5 call O: BN tests + cfg3 bench (bf16 BN apply chunk).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bn.py tests/test_gpu_bf16.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench_bf16.json 2> $OUT/bench_bf16.log
rc=$?; echo "bench bf16 rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_bf16.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/r05n/bench_bf16.json"))["hip_kernels"] if False else None
d = json.load(open("gpurun_out/r05o/bench_bf16.json"))["hip_kernels"]
for k in ("bn_fwd_apply", "bn_bwd_apply", "bn_bwd_reduce", "bn_fwd_stats", "bn_fwd_final"):
    if k in d: print(k, d[k])
PY
