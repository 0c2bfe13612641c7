#!/bin/bash
# Same-box A/B of the current library against tools/_bin/prev.so (tools/build_prev_lib.sh <rev>):
# attention microbenchmarks and C2, alternating. usage: ab_lib_r4.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-ab_lib_r4}
mkdir -p $OUT
export PYTHONPATH=$R
for i in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
    for a in "--batch 2" "--batch 16 --dtype bf16"; do
      timeout -k 10 120 python -u tools/bench_winattn.py $a > $OUT/wa.log 2>&1 || { tail -3 $OUT/wa.log; exit 2; }
      echo "$lib $i $a: $(grep -v amdgpu $OUT/wa.log | tail -1 | cut -c1-120)"
    done
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_${lib}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${lib}_$i.log; exit 4; }
    echo "$lib $i c2 $(tail -1 $OUT/bench_c2_${lib}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["frac"],4), d["roofline"]["avg_launch_ms"])')"
  done
done
