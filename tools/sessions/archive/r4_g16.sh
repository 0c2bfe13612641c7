#!/bin/bash
# Round 4 probe: where the C2 bf16x3 step's critical path is -- default vs bf16 window attention
# (upper bound for a faster attention), serial branches (TSPLAT_STREAMS=0), eager per-stage times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g16}
mkdir -p $OUT
export PYTHONPATH=$R
for v in default attnbf16 serial; do
  case $v in
    default) timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_$v.log 2>&1 ;;
    attnbf16) timeout -k 10 300 python -u bench.py --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_$v.log 2>&1 ;;
    serial) TSPLAT_STREAMS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_$v.log 2>&1 ;;
  esac || { tail -5 $OUT/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/bench_$v.log | cut -c1-120)"
done
timeout -k 10 300 python -u tools/stage_times.py 1 bf16x3 10 > $OUT/stages_x3.log 2>&1 || { tail -5 $OUT/stages_x3.log; exit 2; }
grep -v amdgpu $OUT/stages_x3.log | tail -25
