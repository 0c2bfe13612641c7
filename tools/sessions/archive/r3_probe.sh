#!/bin/bash
# Round-3 probes: per-stage GPU time (C2 and C3), op call sites of the C3 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/probe
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 200 python tools/stage_times.py 1 fp32 10 > $OUT/stages_c2.log 2>&1 || { tail -5 $OUT/stages_c2.log; exit 1; }
grep -v "^{" $OUT/stages_c2.log | grep "gpu"
timeout -k 10 300 python tools/stage_times.py 8 bf16 5 > $OUT/stages_c3.log 2>&1 || { tail -5 $OUT/stages_c3.log; exit 1; }
grep -v "^{" $OUT/stages_c3.log | grep "gpu"
timeout -k 10 300 python tools/op_stacks.py 8 bf16 > $OUT/ops_c3.log 2>&1 || { tail -5 $OUT/ops_c3.log; exit 1; }
head -40 $OUT/ops_c3.log
echo done
