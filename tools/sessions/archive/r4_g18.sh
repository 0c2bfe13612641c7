#!/bin/bash
# Round 4: XCD order in the fp32 Winograd kernels, persistent form out of the bf16x3 auto choice,
# the qkv bias folded into the DINOv2 attention kernel: tests, censuses, C2 (bf16x3 x2, fp32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g18}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_encoder_ops.py tests/test_modules.py -k "wino or mha or depth_anything" -m gpu > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_wino3.py --quick > $OUT/bench_wino3.log 2>&1 || { tail -3 $OUT/bench_wino3.log; exit 2; }
tail -1 $OUT/bench_wino3.log
timeout -k 10 300 python -u tools/bench_wino.py > $OUT/bench_wino_fp32.log 2>&1 || { tail -3 $OUT/bench_wino_fp32.log; exit 3; }
tail -2 $OUT/bench_wino_fp32.log
for v in x3_1 fp32 x3_2; do
  case $v in
    fp32) timeout -k 10 300 python -u bench.py --dense-dtype fp32 --no-cpu-baseline > $OUT/bench_c2_$v.log 2>&1 ;;
    *) timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$v.log 2>&1 ;;
  esac || { tail -5 $OUT/bench_c2_$v.log; exit 4; }
  echo "$v $(tail -1 $OUT/bench_c2_$v.log | cut -c1-120)"
done
