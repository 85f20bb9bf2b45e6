#!/bin/bash
# Round-5 call C: SQ counters of the convbf kernels on one shape (default the
# 64 -> 64 @ 60x80 bs 32 3x3), two --pmc passes (<= 8 SQ counters each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE=${SHAPE:-64,64,60,80,3,1}
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i + 1))
  rm -rf $OUT/p$i
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d "$PWD/$OUT/p$i" -o kp -- \
    python3 tools/convbf_bench.py --only $SHAPE > $OUT/p$i.log 2>&1
  rc=$?
  f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - "$f" <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(convbf_\w+_kernel<[^>]*>)", r["Kernel_Name"])
    if not m:
        continue
    n = m.group(1)
    agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(agg.items()):
    print(f"{n[:60]:60s} " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
PY
done
