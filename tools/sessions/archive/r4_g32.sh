#!/bin/bash
# g32: determinism. bf16x3 encoder module outputs twice with / without deterministic MIOpen solvers;
# run-to-run encoder errors with them; C2 bench deterministic (default now) vs --conv-nondeterministic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g32
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 200 python -u tools/determinism_probe.py bf16x3 1 > $OUT/det_x3_cudnn.log 2>&1 || exit 2
grep -v amdgpu $OUT/det_x3_cudnn.log | cut -c1-200
timeout -k 10 300 python -u tools/encoder_repeat.py 4 --deterministic > $OUT/enc_repeat_det.log 2>&1 || exit 3
grep "encoder vs" $OUT/enc_repeat_det.log
for i in 1 2; do
  for m in det nondet; do
    extra=""; [ $m = nondet ] && extra="--conv-nondeterministic"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $extra > $OUT/bench_c2_${m}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${m}_$i.log; exit 4; }
    echo "$m $i c2 $(tail -1 $OUT/bench_c2_${m}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')"
  done
done
