#!/bin/bash
# Round-5 call J: bf16 pointwise backward timing + SQ counters of its kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/pw_bf16_bench.py > $OUT/pw.log 2>&1; rc=$?; grep -v amdgpu $OUT/pw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/pw_bf16_bench.py --dtype fp32 > $OUT/pw32.log 2>&1; rc=$?; grep -v amdgpu $OUT/pw32.log; [ $rc -eq 0 ] || exit $rc
SHAPE=${SHAPE:-16,8,480,640}
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU"; do
  i=$((i + 1))
  rm -rf $OUT/p$i
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d "$PWD/$OUT/p$i" -o kp -- \
    python3 tools/pw_bf16_bench.py --only $SHAPE > $OUT/p$i.log 2>&1
  rc=$?
  f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - "$f" <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(skip_\w+_kernel<[^>]*>)", r["Kernel_Name"])
    if not m:
        continue
    agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(agg.items()):
    print(f"{n[:70]:70s} " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
PY
done
