#!/bin/bash
# Round 4: C3 lines after the XCD-order changes (fused linears, bf16 conv grid), bf16 conv tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g20}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_e2e.py -k "conv_bf16 or c3" -m gpu > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated.log 2>&1 || { tail -5 $OUT/bench_c3_stated.log; exit 2; }
echo "c3 stated $(tail -1 $OUT/bench_c3_stated.log | cut -c1-120)"
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_bf16dense.log 2>&1 || { tail -5 $OUT/bench_c3_bf16dense.log; exit 3; }
echo "c3 bf16dense $(tail -1 $OUT/bench_c3_bf16dense.log | cut -c1-120)"
timeout -k 10 200 python -u tools/bench_conv_bf16.py > $OUT/bench_conv_bf16.log 2>&1 || { tail -5 $OUT/bench_conv_bf16.log; exit 4; }
tail -8 $OUT/bench_conv_bf16.log
