#!/bin/bash
# g25: fp32 x32 window attention, LDS-DMA form for key-split launches (TSPLAT_WA_DMA=1, default) vs the
# register-staged form (TSPLAT_WA_DMA=0): attention GPU tests, phase stamps, microbenchmark, C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g25
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_encoder_ops.py \
  -k "window_attention or attention_merge" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -2 $OUT/pytest.log
TSPLAT_LIB=tools/_bin/wastamp.so timeout -k 10 120 python -u tools/wa_stamps.py > $OUT/stamps.txt 2>&1 || { tail $OUT/stamps.txt; exit 3; }
grep -v amdgpu $OUT/stamps.txt
for i in 1 2; do
  for d in 0 1; do
    export TSPLAT_WA_DMA=$d
    for a in "--batch 2" "--batch 2 --shift 0"; do
      timeout -k 10 120 python -u tools/bench_winattn.py $a > $OUT/wa.log 2>&1 || { tail -3 $OUT/wa.log; exit 4; }
      echo "dma $d $i $a: $(grep -v amdgpu $OUT/wa.log | tail -1 | cut -c1-120)"
    done
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_${d}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${d}_$i.log; exit 5; }
    echo "dma $d $i c2 $(tail -1 $OUT/bench_c2_${d}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["frac"],4), d["roofline"]["avg_launch_ms"])')"
  done
done
