#!/bin/bash
# g34: which MIOpen kernels the deterministic-solver mode adds to the C2 step (rocprof, --conv-deterministic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/r4_g34
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_det -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --conv-deterministic > $OUT/prof_det.log 2>&1 || exit 1
cd $R
python3 tools/prof_steps.py $OUT/prof_det/run_kernel_trace.csv > $OUT/det_per_step.txt 2>&1
grep -v tsplat $OUT/det_per_step.txt | head -30 | cut -c1-170
