#!/bin/bash
# Round 4: the last two MIOpen 3x3s of the C2 step (256 -> 128 / 64^2 before the bilinear upsample,
# the 64 -> 2 head at 256^2) on the Winograd kernels: tests, C2 bf16x3 x2 and fp32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g19}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_modules.py tests/test_e2e.py tests/test_reference_golden.py tests/test_encoder_ops.py -k "wino or depth_predictor or bf16x3 or encoder or fused_linear or attention_merge or mvt or backbone" -m gpu > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in x3_1 fp32 x3_2; do
  case $v in
    fp32) timeout -k 10 300 python -u bench.py --dense-dtype fp32 --no-cpu-baseline > $OUT/bench_c2_$v.log 2>&1 ;;
    *) timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$v.log 2>&1 ;;
  esac || { tail -5 $OUT/bench_c2_$v.log; exit 4; }
  echo "$v $(tail -1 $OUT/bench_c2_$v.log | cut -c1-120)"
done
