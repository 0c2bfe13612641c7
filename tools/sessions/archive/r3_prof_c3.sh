#!/bin/bash
# C3 (and C2) rocprofv3 kernel-trace per-step summaries plus the C3 op call-site census.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-prof_c3}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python tools/op_stacks.py 8 bf16 > $OUT/ops_c3.log 2>&1 || { tail -5 $OUT/ops_c3.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3.log 2>&1 || { tail -5 $OUT/prof_c3.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c2.log 2>&1 || { tail -5 $OUT/prof_c2.log; exit 1; }
cd $R
python3 tools/prof_steps.py $OUT/prof_c3/run_kernel_trace.csv --skip 2 > $OUT/c3_per_step.txt
python3 tools/prof_steps.py $OUT/prof_c2/run_kernel_trace.csv > $OUT/c2_per_step.txt
head -3 $OUT/c3_per_step.txt; head -3 $OUT/c2_per_step.txt
echo done
