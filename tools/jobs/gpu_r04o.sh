#!/bin/bash
# Round-4 call O: bf16 BN storage vs fp32 kernel (bitwise), Winograd tests
# (restored kernel), then cfg2 A/Bs of Winograd (MDE_WINO) and the
# small-tensor BN kernels (MDE_BN_CHAN), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_bn.py::test_batchnorm_bf16_storage_matches_fp32_kernel" \
  tests/test_gpu_wino.py tests/test_gpu_parity.py -k "bf16_storage or wino or ssim or objective or golden" \
  -q -rfE --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -v "Cannot find the function" $OUT/tests.log | grep -E "^E |FAILED|passed|failed" | head -n 30 | cut -c1-300
[ $rc -le 1 ] || exit $rc
for v in 1 0; do
  MDE_SSIM_PAIR=$v timeout -k 10 300 python3 -u tools/kbench.py --only loss > $OUT/ssim_$v.txt 2>&1
  rc=$?; echo "SSIM_PAIR=$v $(grep ssim3 $OUT/ssim_$v.txt | head -1)"; [ $rc -eq 0 ] || exit $rc
done
ab() {  # name env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > $OUT/ab_$tag.json 2> $OUT/ab_$tag.log
  local rc=$?
  echo "$tag ($*) rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/ab_$tag.json'));print(d['value'],d['ms_per_step'])" 2>&1)"
  return $rc
}
ab base1 MDE_WINO=0 && ab wino1 MDE_WINO=1 && ab base2 MDE_WINO=0 && ab wino2 MDE_WINO=1 && \
  ab nochan1 MDE_WINO=1 MDE_BN_CHAN=0 && ab nochan2 MDE_WINO=1 MDE_BN_CHAN=0
