#!/bin/bash
# SQ instruction / cycle counters of one kernel (regex $1) under a short command ($2...), one
# rocprofv3 --pmc pass per counter group, each under its own time limit; summaries printed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
RE=$1; shift
OUT=$R/gpurun_out/pmck
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
i=0
PGROUPS=${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"}
IFS=';' read -ra GL <<< "$PGROUPS"
for G in "${GL[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex "$RE" -d $OUT/g$i -o run --output-format csv -- "$@" > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/g$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} n={len(v):4d} mean/dispatch={sum(v)/len(v):.4g}")
PY
