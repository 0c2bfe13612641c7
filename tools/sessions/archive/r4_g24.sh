#!/bin/bash
# g24: fp32 x32 window attention with a (batch, window) pair's query blocks and key splits on one XCD
# (TSPLAT_WA_PAIR=1) vs the default order: phase stamps, attention microbenchmark, C2, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g24
mkdir -p $OUT
export PYTHONPATH=$(pwd)
for pr in 0 1; do
  TSPLAT_WA_PAIR=$pr TSPLAT_LIB=tools/_bin/wastamp.so timeout -k 10 120 python -u tools/wa_stamps.py > $OUT/stamps_$pr.txt 2>&1 || exit 2
  echo "== pair $pr"; grep -v amdgpu $OUT/stamps_$pr.txt
done
for i in 1 2; do
  for pr in 0 1; do
    export TSPLAT_WA_PAIR=$pr
    for a in "--batch 2" "--batch 2 --shift 0"; do
      timeout -k 10 120 python -u tools/bench_winattn.py $a > $OUT/wa.log 2>&1 || { tail -3 $OUT/wa.log; exit 3; }
      echo "pair $pr $i $a: $(grep -v amdgpu $OUT/wa.log | tail -1 | cut -c1-120)"
    done
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_${pr}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${pr}_$i.log; exit 4; }
    echo "pair $pr $i c2 $(tail -1 $OUT/bench_c2_${pr}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["frac"],4), d["roofline"]["avg_launch_ms"])')"
  done
done
