#!/bin/bash
# One rocprofv3 --pmc pass over tools/kbench.py (ONLY=groups, PMC="counters") -> per-kernel means.
mkdir -p gpurun_out/kpmc
export TMPDIR=/tmp
rm -rf gpurun_out/kpmc/*
timeout -s KILL 300 rocprofv3 --pmc ${PMC} --output-format csv -d "$PWD/gpurun_out/kpmc" -o kp -- \
  python3 tools/kbench.py --only ${ONLY:-dw} --reps ${REPS:-10} > gpurun_out/kpmc/kbench.log 2>&1
rc=$?
f=$(find gpurun_out/kpmc -name "*counter_collection.csv" | head -1)
echo "pmc rc=$rc file=$f"
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(float.*", "", r["Kernel_Name"]).replace("void mde::(anonymous namespace)::", "")
    key = (n[:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (n, g), cs in sorted(agg.items()):
    print(f"{n:60s} grid {g:>9s} " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
PY
exit $rc
