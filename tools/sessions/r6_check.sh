#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/r6_check; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED|replays vs|bf16x3 vs fp32" $OUT/pytest.log | grep -v "^ " | head -10
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 200 python -u tools/enc_graph_race.py 12 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-120 || exit 1; done
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1; tail -1 $OUT/bench_$i.log | cut -c80-150; done
