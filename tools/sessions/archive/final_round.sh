#!/bin/bash
# Round-end evidence: full GPU tests, smoke, the headline bench (+ rocprof stats, + PMC traffic of
# the dominant kernel), the C3 (batch 8, bf16) and raster-only benches with their profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/final
mkdir -p $OUT
export PYTHONPATH=$R
step() { echo "== $1"; }
# part: "all" (default), "bench" (tests .. raster bench) or "prof" (rocprof passes + PMC)
PART=${1:-all}
if [ "$PART" != "prof" ]; then
step tests
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
step bench
timeout -k 10 500 python bench.py > $OUT/bench_e2e_fp32_b1.log 2>&1 || exit 1
tail -1 $OUT/bench_e2e_fp32_b1.log | cut -c1-200
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
[ "$PART" = "bench" ] && { echo done; exit 0; }
cd /tmp && export TMPDIR=/tmp
step prof
# (rocprof passes without MIOpen's algorithm search, so its trial kernels do not pollute the per-step
# stats; the hand-written kernels are the same launches as in the bench)
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_fp32_b1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_e2e_fp32_b1.log 2>&1 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_raster -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_raster.log 2>&1 || exit 1
if [ "${NO_PMC:-0}" != "1" ]; then
step pmc
cd $R && bash tools/sessions/pmc_round.sh || exit 1
fi
echo done
