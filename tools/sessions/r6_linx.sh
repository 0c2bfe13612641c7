#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/r6_linx; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_e2e.py tests/test_conv.py -m gpu -v --timeout 200 --timeout-method thread -s -k "graph_replays or bf16x3_step_vs or xf32_library" > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|replays vs|bf16x3 vs fp32" $OUT/pytest.log | grep -v "^tests" | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1
TSPLAT_LINX=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_linx1_$i.log 2>&1 || exit 1
done
for f in $OUT/bench_*.log; do echo $f $(tail -1 $f | cut -c1-160); done
