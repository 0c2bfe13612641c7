#!/bin/bash
# Round-5 attention session: x3 / merge tests, microbenchmarks (fp32 vs bf16x3 at b = 2 views), C2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_attn}
mkdir -p $OUT
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_encoder_ops.py -m gpu -q -x -s --timeout 200 --timeout-method thread \
  -k "x3 or attention_merge or window_attention_kernel" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep "x3 attention" $OUT/pytest.log
for d in fp32 x3; do for s in 0 1; do
  timeout -k 10 120 python -u tools/bench_winattn.py --batch 2 --dtype $d --shift $s > $OUT/wa_${d}_$s.log 2>&1 || { tail -5 $OUT/wa_${d}_$s.log; exit 2; }
  grep -v amdgpu $OUT/wa_${d}_$s.log | tail -1
done; done
TAG=$TAG LEGS="cur env" AB_ENV="TSPLAT_ATTN_X3=0" bash tools/sessions/r5_ab.sh
