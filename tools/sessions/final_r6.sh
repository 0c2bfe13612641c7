#!/bin/bash
# Round-6 evidence on the round-end tree. PART = tests | bench | prof | pmc | extra.
#   tests: full GPU suite + smoke; bench: C2 headline (bf16x3, cpu_baseline), C2 exact fp32, C3 as
#   stated, C3 bf16-dense, raster-only; prof: rocprofv3 kernel-trace/stats digests (C2, C3, raster);
#   pmc: FETCH_SIZE / WRITE_SIZE passes (one counter per pass) -> traffic_*.json; extra: determinism
#   probe, replayed-step stage marks, direct-conv census.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-final_r6}
mkdir -p $OUT
export PYTHONPATH=$R
PART=${1:-all}
step() { echo "== $1 $(date +%T)"; }
if [ "$PART" = "all" ] || [ "$PART" = "tests" ]; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 -s > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -2 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -10; exit 1; }
  step smoke
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [ "$PART" = "all" ] || [ "$PART" = "bench" ]; then
  step bench
  timeout -k 10 500 python bench.py > $OUT/bench_e2e_x3_b1.log 2>&1 || { tail -5 $OUT/bench_e2e_x3_b1.log; exit 1; }
  tail -1 $OUT/bench_e2e_x3_b1.log | cut -c1-300
  [ -n "$C2_ONLY" ] && exit 0
  timeout -k 10 500 python bench.py --dense-dtype fp32 --no-cpu-baseline > $OUT/bench_e2e_fp32_b1.log 2>&1 || exit 1
  tail -1 $OUT/bench_e2e_fp32_b1.log | cut -c1-200
  timeout -k 10 500 python bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated.log 2>&1 || exit 1
  tail -1 $OUT/bench_c3_stated.log | cut -c1-200
  timeout -k 10 500 python bench.py --batch 8 --dense-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_bf16dense.log 2>&1 || exit 1
  tail -1 $OUT/bench_c3_bf16dense.log | cut -c1-200
  timeout -k 10 300 python bench.py --workload raster --steps 20 --warmup 3 > $OUT/bench_raster.log 2>&1 || exit 1
  tail -1 $OUT/bench_raster.log | cut -c1-300
fi
if [ "$PART" = "all" ] || [ "$PART" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_x3_b1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_e2e_x3_b1.log 2>&1 || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3_stated -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_c3_stated.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_raster -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_raster.log 2>&1 || exit 1
  cd $R
  for t in e2e_x3_b1 c3_stated raster; do
    python3 tools/prof_steps.py $(find $OUT/prof_$t -name "*kernel_trace.csv" | head -1) > $OUT/${t}_per_step.txt 2>&1 || true
    cp $(find $OUT/prof_$t -name "*kernel_stats.csv" | head -1) $OUT/${t}_kernel_stats.csv
    rm -rf $OUT/prof_$t
  done
  head -30 $OUT/e2e_x3_b1_per_step.txt
fi
if [ "$PART" = "all" ] || [ "$PART" = "pmc" ]; then
  step pmc
  cd /tmp && export TMPDIR=/tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_wa_x3_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $OUT/pmc_wa_x3_$C.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_wa_fp32_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --iters 20 > $OUT/pmc_wa_fp32_$C.log 2>&1 || exit 1
    timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_raster_$C -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 5 --warmup 1 --no-graph --no-cpu-baseline > $OUT/pmc_raster_$C.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_w3_$C -o run --output-format csv -- python3 $R/tools/one_wino3.py 2 163 168 256 256 > $OUT/pmc_w3_$C.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_wa_bf16_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 16 --dtype bf16 --iters 20 > $OUT/pmc_wa_bf16_$C.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_corr_$C -o run --output-format csv -- python3 $R/tools/bench_corr.py --iters 20 > $OUT/pmc_corr_$C.log 2>&1 || exit 1
  done
  cd $R
  f() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
  python3 tools/pmc_traffic.py $(f pmc_wa_x3_FETCH_SIZE) $(f pmc_wa_x3_WRITE_SIZE) win_attn_x3 $OUT/traffic_win_attn_bf16x3_b1.json || true
  python3 tools/pmc_traffic.py $(f pmc_wa_fp32_FETCH_SIZE) $(f pmc_wa_fp32_WRITE_SIZE) win_attn_f32x32 $OUT/traffic_win_attn_fp32_b1.json || true
  python3 tools/pmc_traffic.py $(f pmc_raster_FETCH_SIZE) $(f pmc_raster_WRITE_SIZE) render_kernel,preprocess_kernel,scatter_kernel,zero_kernel $OUT/traffic_raster_fp32_b1.json || true
  python3 tools/pmc_traffic.py $(f pmc_w3_FETCH_SIZE) $(f pmc_w3_WRITE_SIZE) conv_kernel $OUT/traffic_wino3_163x168_b1.json || true
  python3 tools/pmc_traffic.py $(f pmc_wa_bf16_FETCH_SIZE) $(f pmc_wa_bf16_WRITE_SIZE) win_attn_bf16_v3 $OUT/traffic_win_attn_bf16_b8.json || true
  python3 tools/pmc_traffic.py $(f pmc_corr_FETCH_SIZE) $(f pmc_corr_WRITE_SIZE) uv_coarse $OUT/traffic_uv_coarse_fp32_b1.json || true
  for d in pmc_wa_x3_FETCH_SIZE pmc_wa_x3_WRITE_SIZE pmc_wa_fp32_FETCH_SIZE pmc_wa_fp32_WRITE_SIZE pmc_raster_FETCH_SIZE pmc_raster_WRITE_SIZE pmc_w3_FETCH_SIZE pmc_w3_WRITE_SIZE pmc_wa_bf16_FETCH_SIZE pmc_wa_bf16_WRITE_SIZE pmc_corr_FETCH_SIZE pmc_corr_WRITE_SIZE; do rm -rf $OUT/$d; done
  ls $OUT/*.json
fi
if [ "$PART" = "cache" ]; then
  step cache
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_corr_cache -o run --output-format csv -- python3 $R/tools/bench_corr.py --iters 20 > $OUT/pmc_corr_cache.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD -d $OUT/pmc_corr_sq -o run --output-format csv -- python3 $R/tools/bench_corr.py --iters 20 > $OUT/pmc_corr_sq.log 2>&1 || exit 1
  cd $R
  python3 - $OUT <<'PY'
import csv, glob, sys, collections
for tag in ("pmc_corr_cache", "pmc_corr_sq"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "uv_coarse" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{tag} {k:28s} n={len(v):4d} mean/dispatch={sum(v)/len(v):.4g}")
PY
  rm -rf $OUT/pmc_corr_cache $OUT/pmc_corr_sq
fi
if [ "$PART" = "all" ] || [ "$PART" = "extra" ]; then
  step extra
  timeout -k 10 300 python -u tools/determinism_probe.py bf16x3 0 > $OUT/determinism_bf16x3.log 2>&1 || { tail -5 $OUT/determinism_bf16x3.log; exit 1; }
  tail -3 $OUT/determinism_bf16x3.log
  timeout -k 10 300 python -u tools/graph_stages.py > $OUT/stages_c2.log 2>&1 || exit 1
  grep -v amdgpu $OUT/stages_c2.log | head -25
  timeout -k 10 300 python -u tools/direct_census.py > $OUT/direct_census.log 2>&1 || exit 1
  tail -1 $OUT/direct_census.log
fi
echo done
