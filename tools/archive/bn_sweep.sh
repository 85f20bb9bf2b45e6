#!/bin/bash
mkdir -p gpurun_out
export COLD=1 SHAPES="64,60,80;128,30,40;32,120,160;256,15,20;16,240,320"
for cfg in "2048 4096" "1024 4096" "512 4096" "1024 8192" "512 16384" "4096 2048"; do
  set -- $cfg
  echo "== target $1 minslice $2"
  MDE_BN_TARGET=$1 MDE_BN_MINSLICE=$2 timeout -k 10 120 python tools/bn_bench.py || exit $?
done
