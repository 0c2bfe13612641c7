#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
OUT=gpurun_out/r4_g9
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > $OUT/pytest_w3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_w3.log | head; tail -3 $OUT/pytest_w3.log; exit 1; }
tail -1 $OUT/pytest_w3.log
timeout -k 10 200 python -u tools/ab_w3_n.py > $OUT/ab_w3_n.log 2>&1 || exit 4
grep -v amdgpu $OUT/ab_w3_n.log
timeout -k 10 400 python -u tools/bench_wino3.py > $OUT/bench_wino3.log 2>&1 || { tail -3 $OUT/bench_wino3.log; exit 2; }
grep -v amdgpu $OUT/bench_wino3.log
