#!/bin/bash
# Round 4: Winograd 32x32 forms with the next chunk's transform beside the MFMAs (PT): kernel tests,
# census (forms), phase clocks, e2e bf16x3 test, C2 x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g15}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > $OUT/pytest_w3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_w3.log | head; tail -3 $OUT/pytest_w3.log; exit 1; }
tail -1 $OUT/pytest_w3.log
timeout -k 10 400 python -u tools/bench_wino3.py > $OUT/bench_wino3.log 2>&1 || { tail -3 $OUT/bench_wino3.log; exit 2; }
grep -v amdgpu $OUT/bench_wino3.log | tail -26
TSPLAT_LIB=tools/_bin/w3stamp.so timeout -k 10 120 python -u tools/w3_stamps.py > $OUT/w3_stamps.log 2>&1 || { tail -5 $OUT/w3_stamps.log; exit 3; }
grep -v amdgpu $OUT/w3_stamps.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_e2e.py -k "bf16x3" -m gpu > $OUT/pytest_e2e.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_e2e.log | head; tail -3 $OUT/pytest_e2e.log; exit 4; }
tail -1 $OUT/pytest_e2e.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$i.log 2>&1 || { tail -5 $OUT/bench_c2_$i.log; exit 5; }
  echo "c2 $i $(tail -1 $OUT/bench_c2_$i.log | cut -c1-120)"
done
