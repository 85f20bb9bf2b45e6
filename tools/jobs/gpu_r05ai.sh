#!/bin/bash
# Round-5 call AI: Winograd XCD split for the weight-heavy NewCRF projections:
# parity, per-shape timing with and without the split, FETCH_SIZE of both,
# cfg4 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r05ai
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -q -rfE -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $OUT/t.log | tail -3 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
for xs in 0 1; do
  echo "== MDE_WINO_XSPLIT=$xs"
  MDE_WINO_XSPLIT=$xs timeout -k 10 200 python3 -u tools/wino_bench.py --newcrf > $OUT/wb_$xs.log 2>&1
  rc=$?; grep wino $OUT/wb_$xs.log; [ $rc -eq 0 ] || exit $rc
  MDE_WINO_XSPLIT=$xs timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/pmc_$xs" -o f -- python3 tools/wino_bench.py --newcrf --reps 3 > $OUT/pmc_$xs.log 2>&1
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for xs in 0 1; do
  MDE_WINO_XSPLIT=$xs timeout -k 10 300 python3 -u bench.py --workload newcrf --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench_$xs.json 2> $OUT/bench_$xs.log
  rc=$?; echo "bench xsplit=$xs rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$xs.json'));k=d['hip_kernels'];print(d['value'], d['ms_per_step'], [(n, k[n]['ms_per_step']) for n in k if n.startswith('wino')])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
