#!/bin/bash
# Round-5 coarse-correlation probe: the dedup kernel stopped after each phase (TSPLAT_CORR_DIAG =
# 1 marks, 2 + rank, 3 + dots, 0 full) at the production 64^2 b = 1 shape, and the variant knob.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_corr}
mkdir -p $OUT
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
for d in 1 2 3 0; do
  TSPLAT_CORR_DIAG=$d timeout -k 10 120 python -u tools/bench_corr.py --iters 200 > $OUT/diag$d.log 2>&1 || exit 1
  echo "diag $d: $(tail -1 $OUT/diag$d.log)"
done
for v in ${VARIANTS:-}; do
  TSPLAT_UV_COARSE_VARIANT=$v timeout -k 10 120 python -u tools/bench_corr.py --iters 200 > $OUT/var$v.log 2>&1 || exit 1
  echo "variant $v: $(tail -1 $OUT/var$v.log)"
done
