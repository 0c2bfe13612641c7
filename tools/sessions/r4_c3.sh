#!/bin/bash
# Round 4: config C3 (BASELINE.json configs[2]: batch 8, bf16 attention + fp32 raster) as stated --
# dense layers bf16x3 (>= the reference's TF32), window attention bf16 -- and the narrower
# bf16-dense variant, each with a rocprofv3 kernel trace (per-step digest by tools/prof_steps.py);
# then the stated-mode GPU test against the fp32 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_c3}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 > $OUT/bench_c3_stated.log 2>&1 || { tail -5 $OUT/bench_c3_stated.log; exit 1; }
echo "stated $(tail -1 $OUT/bench_c3_stated.log | cut -c1-200)"
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16 > $OUT/bench_c3_bf16dense.log 2>&1 || { tail -5 $OUT/bench_c3_bf16dense.log; exit 1; }
echo "bf16-dense $(tail -1 $OUT/bench_c3_bf16dense.log | cut -c1-200)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3_stated -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3_stated.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3_bf16dense -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3_bf16dense.log 2>&1 || exit 3
cd $R
for t in stated bf16dense; do
  python3 tools/prof_steps.py $OUT/prof_c3_$t/run_kernel_trace.csv > $OUT/c3_${t}_per_step.txt 2>&1 || true
  head -12 $OUT/c3_${t}_per_step.txt
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_e2e.py -k "c3" -m gpu > $OUT/pytest_c3.log 2>&1 || { tail -20 $OUT/pytest_c3.log; exit 4; }
grep -E "PSNR|passed|failed" $OUT/pytest_c3.log | tail -8
