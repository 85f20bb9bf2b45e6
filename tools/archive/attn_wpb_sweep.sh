#!/bin/bash
# Window-attention windows-per-block sweep (MDE_ATTN_FWD_WPB / MDE_ATTN_BWD_WPB; 0 = the built-in rule).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VALS:-0 1 2 3 4 6 9 0}; do
  MDE_ATTN_FWD_WPB=$v MDE_ATTN_BWD_WPB=$v timeout -k 10 300 python -u tools/kbench.py --only attn > gpurun_out/wpb_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/wpb_$v.log; exit $rc; }
  echo "== wpb $v"; grep "s0 " gpurun_out/wpb_$v.log
done
