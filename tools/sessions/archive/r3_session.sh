#!/bin/bash
# Round-3 GPU session: GPU tests (or a subset), smoke, the e2e / raster benches, the 2-rank
# self-launched bench on one GPU (gloo), optional rocprof pass. Stops at the first fault / timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
TAG=${TAG:-s1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONPATH=$R
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no fault)
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v -rA -s --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  ok $rc || exit $rc
fi
if [ "${RUN_SMOKE:-1}" = 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_e2e.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $OUT/bench_e2e.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_RASTER:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --workload raster --steps 20 --warmup 3 > $OUT/bench_raster.log 2>&1; rc=$?
  echo "raster rc=$rc"; tail -1 $OUT/bench_raster.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_MULTI:-0}" = 1 ]; then
  TSPLAT_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_gpus2_gloo.log 2>&1; rc=$?
  echo "gpus2 rc=$rc"; grep '^{' $OUT/bench_gpus2_gloo.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python3 $R/bench.py ${PROF_ARGS:-} --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof.log 2>&1; rc=$?
  echo "prof rc=$rc"; tail -2 $OUT/prof.log
  [ $rc -eq 0 ] || exit $rc
fi
echo done
