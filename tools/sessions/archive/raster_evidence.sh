#!/bin/bash
# Rasterizer evidence: GPU tests, raster-only bench line, rocprof kernel stats + steady-state
# per-step breakdown (profiles/<tag>/raster_only_*), phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
TAG=${TAG:-r2}
OUT=$R/gpurun_out/raster_$TAG
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload raster --steps 20 --warmup 3 > $OUT/bench_raster.log 2>&1 || exit 1
tail -1 $OUT/bench_raster.log | cut -c1-300
timeout -k 10 120 python tools/bench_raster.py --diag 0,2 > $OUT/phases.log 2>&1 || exit 1
cat $OUT/phases.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
echo done
