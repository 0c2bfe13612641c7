#!/bin/bash
# Round-5 coarse-correlation A/B: the dedup kernel's register budget for 5 vs 6 waves per SIMD
# (TSPLAT_CORR_WPE) on tools/bench_corr.py (production 64^2 b = 1 and b = 8), alternating, after the
# kernel's tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_corrab}
mkdir -p $OUT
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops.py tests/test_reference_golden.py -m gpu -q -x -k "coarse or uv" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for lib in 5 6; do
    export TSPLAT_CORR_WPE=$lib
    for b in 1 8; do
      timeout -k 10 120 python -u tools/bench_corr.py --batch $b --iters 300 > $OUT/${lib}_b${b}_$i.log 2>&1 || exit 1
      echo "$lib b=$b run $i: $(tail -1 $OUT/${lib}_b${b}_$i.log)"
    done
  done
done
