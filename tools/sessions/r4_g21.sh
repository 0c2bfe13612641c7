#!/bin/bash
# Round 4: packed softmax arithmetic (v_pk_fma / v_pk_add, v_max3 tree) in the fp32 x32 and bf16 v3
# window-attention kernels: attention tests, microbenchmarks, C2 x2, C3 stated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g21}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_encoder_ops.py tests/test_modules.py -k "window or attention or mvt or backbone" -m gpu > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for a in "--batch 2" "--batch 2 --shift 0" "--batch 16 --dtype bf16" "--batch 16 --dtype bf16 --shift 0"; do
  timeout -k 10 120 python -u tools/bench_winattn.py $a > $OUT/wa.log 2>&1 || { tail -3 $OUT/wa.log; exit 2; }
  echo "$a: $(grep -v amdgpu $OUT/wa.log | tail -2 | tr '\n' ' ' | cut -c1-200)"
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$i.log 2>&1 || { tail -5 $OUT/bench_c2_$i.log; exit 4; }
  echo "c2 $i $(tail -1 $OUT/bench_c2_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["roofline"]["achieved"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])')"
done
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated.log 2>&1 || { tail -5 $OUT/bench_c3_stated.log; exit 5; }
echo "c3 stated $(tail -1 $OUT/bench_c3_stated.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["roofline"]["achieved"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])')"
