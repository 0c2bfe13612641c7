#!/bin/bash
# x3 attention A/B: phase clocks and microbench for TSPLAT_X3_XORDER 0 / 1; optional C2 legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_x3ab}
mkdir -p $OUT
export PYTHONPATH=$R
for xo in 0 1; do
  TSPLAT_X3_XORDER=$xo TSPLAT_LIB=tools/_bin/wastamp.so timeout -k 10 120 python -u tools/wa_stamps.py --x3 > $OUT/stamps_x3_$xo.log 2>&1 || { tail -5 $OUT/stamps_x3_$xo.log; exit 1; }
  echo "xorder $xo"; grep -v amdgpu $OUT/stamps_x3_$xo.log | head -4
  for s in 0 1; do
    TSPLAT_X3_XORDER=$xo timeout -k 10 120 python -u tools/bench_winattn.py --batch 2 --dtype x3 --shift $s > $OUT/wa_$xo_$s.log 2>&1 || exit 2
    echo "xorder $xo shift $s: $(grep -v amdgpu $OUT/wa_$xo_$s.log | tail -1)"
  done
done
if [ -n "$C2" ]; then TAG=$TAG LEGS="cur env" AB_ENV="$C2" bash tools/sessions/r5_ab.sh; fi
