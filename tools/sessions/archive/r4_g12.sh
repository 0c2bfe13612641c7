#!/bin/bash
# Round 4: pipelined bf16x3 GEMM (LDS-DMA ring) -- kernel tests, GEMM shapes vs hipBLASLt, the xf32
# probe with mm / 3-D matmul variants, then a C2 A/B with the GEMM dispatched (TSPLAT_LIN3=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g12}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv.py -k "linear_bf16x3" -m gpu > $OUT/pytest_lin3.log 2>&1 || { grep -E "FAILED|Error|rel err" $OUT/pytest_lin3.log | head; tail -3 $OUT/pytest_lin3.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_lin3.log | tail -1
timeout -k 10 200 python -u tools/bench_split_gemm.py > $OUT/split_gemm.log 2>&1 || { tail -3 $OUT/split_gemm.log; exit 2; }
grep -v amdgpu $OUT/split_gemm.log | cut -c1-230
timeout -k 10 120 python -u tools/bench_xf32.py --allow-tf32 > $OUT/xf32_tf32.log 2>&1 || { tail -3 $OUT/xf32_tf32.log; exit 3; }
grep -v amdgpu $OUT/xf32_tf32.log | cut -c1-230
for i in 1 2; do
  for l in 0 1; do
    TSPLAT_LIN3=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_lin${l}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_lin${l}_$i.log; exit 4; }
    echo "lin3=$l $i $(tail -1 $OUT/bench_c2_lin${l}_$i.log | cut -c1-120)"
  done
done
