#!/bin/bash
# Round-5 call F: convbf parity (+ epilogue statistics), the bf16 / fp32 step
# goldens and graph-DP tests after routing DDRNet's BN statistics through the
# conv epilogues, per-shape timing, cfg3 / cfg2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|no tests ran|Error|error:" $OUT/$name.log | tail -n 12 | cut -c1-300
  return $rc
}
run convbf 600 python3 -u -m pytest tests/test_gpu_convbf.py -q -rfE -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
run models 900 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_graph_dp.py tests/test_gpu_parity.py tests/test_gpu_graph.py -q -rfE -p no:cacheprovider --timeout 600 --timeout-method thread || exit 1
run kbench 300 python3 -u tools/convbf_bench.py && grep -v amdgpu.ids $OUT/kbench.log | cut -c1-150 || exit 1
for cfg in bf16 fp32; do
  a=""; [ $cfg = bf16 ] && a="--amp bf16"
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $a --steps 30 --warmup 5 > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.log
  rc=$?; echo "bench $cfg rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05f/bench_bf16.json"))
ks = sorted(d["hip_kernels"].items(), key=lambda kv: -kv[1]["ms_per_step"])[:30]
for k, v in ks:
    print(f"{k:28s} {v['ms_per_step']:7.3f} ms/step {v['launches']:5d} launches {v.get('GBps', '')} GB/s {v.get('TFLOPs', '')}")
PY
