#!/bin/bash
# rocprofv3 kernel trace + stats of tools/kbench.py (ONLY=groups) -> gpurun_out/kprof/
mkdir -p gpurun_out/kprof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/kprof" -o kb -- \
  python3 tools/kbench.py --only ${ONLY:-dw} --reps ${REPS:-20} > gpurun_out/kprof/kbench.log 2>&1
rc=$?
f=$(find gpurun_out/kprof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us avg {int(r["Calls"]):6d} calls  {r["Name"][:150]}')
PY
exit $rc
