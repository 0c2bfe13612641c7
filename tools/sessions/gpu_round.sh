#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprof. Stops at the first GPU fault/timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${TAG:-r1}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no fault)
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -m pytest ${PYTEST_TARGET:-tests} -m gpu -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu_$TAG.log
  ok $rc || exit $rc
fi
if [ "${RUN_SMOKE:-1}" = 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 $OUT/smoke_$TAG.log
  ok $rc || exit $rc
fi
if [ "${RUN_BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -3 $OUT/bench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
      python3 $R/bench.py ${BENCH_ARGS:-} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1; rc=$?
  echo "prof rc=$rc"; tail -3 $OUT/prof_$TAG.log
  find $OUT/prof_$TAG -name "*stats*" | head
fi
if [ "${RUN_PMC:-0}" = 1 ]; then
  # HBM traffic of the dominant kernel: FETCH_SIZE and WRITE_SIZE in separate passes (eager launches)
  cd /tmp && export TMPDIR=/tmp
  DOM=${PMC_KERNEL:-win_attn}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C -d $OUT/pmc_${TAG}_$C -o run --output-format csv -- \
        python3 $R/bench.py ${BENCH_ARGS:-} --steps 3 --warmup 1 --no-graph --no-cpu-baseline --dominant $DOM > $OUT/pmc_${TAG}_$C.log 2>&1; rc=$?
    echo "pmc $C rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
