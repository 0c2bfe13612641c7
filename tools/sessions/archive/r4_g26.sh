#!/bin/bash
# g26: fresh C2 (bf16x3 dense) rocprof kernel trace + per-step digest, to rank what is left.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/r4_g26
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_x3_b1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_e2e_x3_b1.log 2>&1 || exit 1
cd $R
python3 tools/prof_steps.py $OUT/prof_e2e_x3_b1/run_kernel_trace.csv > $OUT/e2e_x3_b1_per_step.txt 2>&1
head -45 $OUT/e2e_x3_b1_per_step.txt | cut -c1-150
