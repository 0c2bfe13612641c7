#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one counter per pass) of the hand-written kernels the
# bench's roofline objects name: window attention fp32 (B = 2 views, the C2 shape), bf16 (B = 16,
# the C3 shape) and the raster-only workload. Short programs, each pass under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== $C attention fp32 b2"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/wa_fp32_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --iters 20 > $OUT/wa_fp32_$C.log 2>&1 || exit 1
  echo "== $C attention bf16 b16"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/wa_bf16_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 16 --dtype bf16 --iters 20 > $OUT/wa_bf16_$C.log 2>&1 || exit 1
  echo "== $C raster"
  timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/raster_$C -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 5 --warmup 1 --no-graph --no-cpu-baseline > $OUT/raster_$C.log 2>&1 || exit 1
done
echo done
