#!/bin/bash
# Round 4: C2 A/B (exact fp32 vs bf16x3 dense), alternating, then a rocprofv3 kernel trace of the
# bf16x3 C2 step (per-step digest by tools/prof_steps.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g4}
mkdir -p $OUT
export PYTHONPATH=$R
for i in 1 2; do
  for d in fp32 bf16x3; do
    timeout -k 10 300 python -u bench.py --dense-dtype $d --no-cpu-baseline > $OUT/bench_c2_${d}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${d}_$i.log; exit 1; }
    echo "$d $i $(tail -1 $OUT/bench_c2_${d}_$i.log | cut -c1-160)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_x3 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c2_x3.log 2>&1 || exit 2
cd $R
python3 tools/prof_steps.py $OUT/prof_c2_x3/run_kernel_trace.csv > $OUT/c2_x3_per_step.txt 2>&1 || true
python3 tools/overlap_report.py $OUT/prof_c2_x3/run_kernel_trace.csv > $OUT/c2_x3_overlap.txt 2>&1 || true
head -45 $OUT/c2_x3_per_step.txt; tail -8 $OUT/c2_x3_overlap.txt
