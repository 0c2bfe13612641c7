#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export PYTHONPATH=$R
OUT=$R/gpurun_out/r6_dpt; mkdir -p $OUT
timeout -k 10 200 python tools/dpt_prof.py 50 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/tools/dpt_prof.py 20 > $OUT/prof.log 2>&1 || exit 1
cd $R
python3 tools/prof_steps.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/per_step.txt 2>&1
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e3/22:.1f} us per call (22 calls)")
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e3/22:8.1f} us/call  n/call={int(r["Calls"])/22:5.1f} avg={float(r["AverageNs"])/1e3:6.1f}  {r["Name"][:110]}')
PY
rm -rf $OUT/prof
