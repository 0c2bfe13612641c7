#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
OUT=gpurun_out/r4_g8
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > $OUT/pytest_w3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_w3.log | head; tail -3 $OUT/pytest_w3.log; exit 1; }
tail -1 $OUT/pytest_w3.log
timeout -k 10 300 python -u tools/bench_wino3.py --quick > $OUT/bench_wino3.log 2>&1 || { tail -3 $OUT/bench_wino3.log; exit 2; }
grep -v amdgpu $OUT/bench_wino3.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$i.log 2>&1 || exit 3
  echo "c2 $i $(tail -1 $OUT/bench_c2_$i.log | cut -c90-140)"
done
timeout -k 10 200 python -u tools/ab_w3_n.py > $OUT/ab_w3_n.log 2>&1 || exit 4
grep -v amdgpu $OUT/ab_w3_n.log
