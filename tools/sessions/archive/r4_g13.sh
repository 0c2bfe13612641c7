#!/bin/bash
# Round 4: bf16x3 mode's library linears on hipBLASLt's emulated-xf32 GEMM (kernels.linear_xf32):
# kernel-level accuracy, DINOv2 / e2e bf16x3 tests, C2 A/B (TSPLAT_LINX=0/1), C3 stated with it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g13}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv.py tests/test_modules.py tests/test_e2e.py -k "linear_xf32 or depth_anything or bf16x3_step" -m gpu -s > $OUT/pytest_linx.log 2>&1 || { grep -E "FAILED|Error|rel err" $OUT/pytest_linx.log | head; tail -3 $OUT/pytest_linx.log; exit 1; }
grep -E "rel err|passed|failed" $OUT/pytest_linx.log | tail -8
for i in 1 2; do
  for l in 0 1; do
    TSPLAT_LINX=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_linx${l}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_linx${l}_$i.log; exit 4; }
    echo "linx=$l $i $(tail -1 $OUT/bench_c2_linx${l}_$i.log | cut -c1-120)"
  done
done
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated_linx.log 2>&1 || { tail -5 $OUT/bench_c3_stated_linx.log; exit 5; }
echo "c3 stated linx=1 $(tail -1 $OUT/bench_c3_stated_linx.log | cut -c1-120)"
