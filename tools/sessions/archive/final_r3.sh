#!/bin/bash
# Round-3 end evidence: full GPU tests, smoke, benches (C2 headline with cpu_baseline, C3, b8 fp32,
# raster-only), rocprof kernel-trace/stats of C2 / C3 / raster, PMC FETCH_SIZE / WRITE_SIZE passes
# (one counter per pass) digested into traffic_*.json. PART = tests | bench | prof | all.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-final_r3}
mkdir -p $OUT
export PYTHONPATH=$R
PART=${1:-all}
step() { echo "== $1 $(date +%T)"; }
if [ "$PART" = "all" ] || [ "$PART" = "tests" ]; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -2 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -10; exit 1; }
  step smoke
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [ "$PART" = "all" ] || [ "$PART" = "bench" ]; then
  step bench
  timeout -k 10 500 python bench.py > $OUT/bench_e2e_fp32_b1.log 2>&1 || { tail -5 $OUT/bench_e2e_fp32_b1.log; exit 1; }
  tail -1 $OUT/bench_e2e_fp32_b1.log | cut -c1-300
  step c3
  timeout -k 10 500 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_bf16_b8.log 2>&1 || exit 1
  tail -1 $OUT/bench_c3_bf16_b8.log | cut -c1-200
  step b8fp32
  timeout -k 10 500 python bench.py --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_fp32_b8.log 2>&1 || exit 1
  tail -1 $OUT/bench_fp32_b8.log | cut -c1-200
  step raster
  timeout -k 10 300 python bench.py --workload raster --steps 20 --warmup 3 > $OUT/bench_raster.log 2>&1 || exit 1
  tail -1 $OUT/bench_raster.log | cut -c1-200
fi
if [ "$PART" = "all" ] || [ "$PART" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_fp32_b1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_e2e_fp32_b1.log 2>&1 || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_raster -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_raster.log 2>&1 || exit 1
  cd $R
  for t in e2e_fp32_b1 c3 raster; do python3 tools/prof_steps.py $OUT/prof_$t/run_kernel_trace.csv > $OUT/${t}_per_step.txt 2>&1 || true; done
  step pmc
  cd /tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_wa_fp32_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --iters 20 > $OUT/pmc_wa_fp32_$C.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_wa_bf16_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 16 --dtype bf16 --iters 20 > $OUT/pmc_wa_bf16_$C.log 2>&1 || exit 1
    timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_raster_$C -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 5 --warmup 1 --no-graph --no-cpu-baseline > $OUT/pmc_raster_$C.log 2>&1 || exit 1
  done
  cd $R
  f() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
  python3 tools/pmc_traffic.py $(f pmc_wa_fp32_FETCH_SIZE) $(f pmc_wa_fp32_WRITE_SIZE) win_attn_f32x32 $OUT/traffic_win_attn_fp32_b1.json || true
  python3 tools/pmc_traffic.py $(f pmc_wa_bf16_FETCH_SIZE) $(f pmc_wa_bf16_WRITE_SIZE) win_attn_bf16 $OUT/traffic_win_attn_bf16_b8.json || true
  python3 tools/pmc_traffic.py $(f pmc_raster_FETCH_SIZE) $(f pmc_raster_WRITE_SIZE) render_kernel,preprocess_kernel,scan_kernel,scatter_kernel,zero_kernel $OUT/traffic_raster_fp32_b1.json || true
  ls $OUT/*.json
fi
echo done
