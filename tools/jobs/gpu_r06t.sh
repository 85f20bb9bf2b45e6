#!/bin/bash
# Round 6 T: vendor GEMM selection for cfg4's forward / data-gradient GEMMs:
# hipBLASLt (default) vs rocBLAS, and PyTorch TunableOp (tune once, then replay the table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06t}
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --workload newcrf --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $OUT/bench_$tag.json 2> $OUT/bench_$tag.log
  local rc=$?; echo "bench $tag: $(head -c 200 $OUT/bench_$tag.json)"; [ $rc -eq 0 ] || exit $rc
}
b lt TORCH_BLAS_PREFER_HIPBLASLT=1
b rb TORCH_BLAS_PREFER_HIPBLASLT=0
b tune PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30
ls -la $OUT/
b tuned PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop.csv
b lt2 TORCH_BLAS_PREFER_HIPBLASLT=1
