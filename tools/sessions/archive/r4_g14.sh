#!/bin/bash
# Round 4: the fused transformer linears in bf16x3 (tsplat_linear_f32_fwd flag 256): kernel tests in
# both dense modes, module / e2e bf16x3 tests, C2 A/B (TSPLAT_LINF3=0/1), C3 stated with it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g14}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_encoder_ops.py tests/test_modules.py tests/test_e2e.py -k "fused_linear or attention_merge or bf16x3 or mvt or backbone or uv" -m gpu > $OUT/pytest_linf3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_linf3.log | head; tail -3 $OUT/pytest_linf3.log; exit 1; }
tail -1 $OUT/pytest_linf3.log
for i in 1 2; do
  for l in 0 1; do
    TSPLAT_LINF3=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_linf3${l}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_linf3${l}_$i.log; exit 4; }
    echo "linf3=$l $i $(tail -1 $OUT/bench_c2_linf3${l}_$i.log | cut -c1-120)"
  done
done
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated.log 2>&1 || { tail -5 $OUT/bench_c3_stated.log; exit 5; }
echo "c3 stated $(tail -1 $OUT/bench_c3_stated.log | cut -c1-120)"
