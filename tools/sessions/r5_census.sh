#!/bin/bash
# Round-5 census: the bf16x3 Winograd launches and the fused linears of one eager step at b = 1
# (C2) and b = 8 (C3 as stated), per shape with HIP-event times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_census}
mkdir -p $OUT
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 200 python -u tools/wino_census.py bf16x3 1 > $OUT/wino_b1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wino_census.py bf16x3 8 > $OUT/wino_b8.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/linear_census.py bf16x3 1 > $OUT/linear_b1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/linear_census.py bf16x3 8 > $OUT/linear_b8.log 2>&1 || exit 1
tail -3 $OUT/*.log
