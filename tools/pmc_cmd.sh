#!/bin/bash
# One rocprofv3 --pmc pass (PMC="counters") over an arbitrary python command
# (ARGS = the script and its arguments, run as `python3 $ARGS`), summarised
# per kernel: mean counter value per dispatch and dispatch count.
#   PMC=FETCH_SIZE TAG=wg ARGS="tools/wgrad_bench.py" bash tools/pmc_cmd.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/pmc_${TAG:-x}_${PMC// /_}
rm -rf "$D"; mkdir -p "$D"
export TMPDIR=/tmp
timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc ${PMC} --output-format csv -d "$PWD/$D" -o p -- \
  python3 ${ARGS} > "$D/run.log" 2>&1
rc=$?
f=$(find "$D" -name "*counter_collection.csv" | head -1)
echo "pmc ${TAG:-x} ${PMC} rc=$rc"
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    key = (n[:90], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (n, g), cs in sorted(agg.items()):
    print(f"{n:90s} grid {g:>9s} " + " ".join(f"{c}={sum(v)/len(v):.5g} (n={len(v)})" for c, v in sorted(cs.items())))
PY
exit $rc
