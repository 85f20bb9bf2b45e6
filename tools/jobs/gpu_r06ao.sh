#!/bin/bash
# Round 6 AO: per-shape wide weight-gradient times (incl. reduction) vs forced block counts,
# NewCRF projection shapes (bs 16) and DDRNet shapes (bs 32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06ao}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 0 384 768 1024; do
  if [ $b = 0 ]; then e=""; else e="MDE_WIDE_BLOCKS=$b"; fi
  env $e timeout -k 10 200 python3 -u tools/wgrad_bench.py --newcrf > $OUT/nc_$b.txt 2>&1
  rc=$?; echo "== newcrf blocks=$b rc=$rc"; grep "wgrad" $OUT/nc_$b.txt | sed 's/MIOpen.*//'; [ $rc -eq 0 ] || exit $rc
done
for b in 0 768; do
  if [ $b = 0 ]; then e=""; else e="MDE_WIDE_BLOCKS=$b"; fi
  env $e timeout -k 10 300 python3 -u tools/wgrad_bench.py > $OUT/gd_$b.txt 2>&1
  rc=$?; echo "== ddrnet blocks=$b rc=$rc"; grep "^\[wpb" $OUT/gd_$b.txt | sed 's/MIOpen.*//'; [ $rc -eq 0 ] || exit $rc
done
