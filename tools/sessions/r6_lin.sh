#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/r6_lin; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAILED|golden.*bf16x3" $OUT/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/op_stacks.py 1 bf16x3 2>&1 | grep -E ' (mm|addmm|bmm|baddbmm|linear|matmul) '
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1; tail -1 $OUT/bench_$i.log | cut -c1-150; done
