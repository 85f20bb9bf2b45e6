#!/bin/bash
# Round-5 call Y: convbf 2D-patch epilogue through LDS (row segments): tests, per-shape kernels, cfg3 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_convbf.py tests/test_gpu_bf16.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/convbf_bench.py > $OUT/kb.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/kb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --amp bf16 --steps 30 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('convbf')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
