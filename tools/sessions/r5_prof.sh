#!/bin/bash
# Round-5 per-step kernel digest of a bench configuration: rocprofv3 kernel-trace/stats (CSV), then
# tools/prof_steps.py -> <name>_per_step.txt. usage: TAG=<tag> NAME=e2e_x3_b1 ARGS="" bash tools/sessions/r5_prof.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_prof}
mkdir -p $OUT
export PYTHONPATH=$R
NAME=${NAME:-e2e_x3_b1}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_$NAME -o run --output-format csv -- python3 $R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${ARGS} > $OUT/prof_$NAME.log 2>&1 || { tail -5 $OUT/prof_$NAME.log; exit 1; }
cd $R
python3 tools/prof_steps.py $(find $OUT/prof_$NAME -name "*kernel_trace.csv" | head -1) ${GRIDS:+--grids $GRIDS} ${TIMELINE:+--timeline $OUT/${NAME}_timeline.txt} > $OUT/${NAME}_per_step.txt 2>&1
cp $(find $OUT/prof_$NAME -name "*kernel_stats.csv" | head -1) $OUT/${NAME}_kernel_stats.csv
rm -rf $OUT/prof_$NAME
head -45 $OUT/${NAME}_per_step.txt
tail -1 $OUT/prof_$NAME.log | cut -c1-200
