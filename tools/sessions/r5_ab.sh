#!/bin/bash
# Round-5 same-box A/B: tests of the changed kernels, then the current library vs tools/_bin/prev.so
# (tools/build_prev_lib.sh <rev>) on the Winograd census and C2, alternating; extra env A/Bs via
# AB_ENV ("NAME=VALUE" applied to the 'env' leg, run against the current library).
# usage: TAG=<tag> TESTS="tests/test_conv.py" AB_ENV="TSPLAT_CONV_ZSPLIT=0" bash tools/sessions/r5_ab.sh
# (LEGS="cur env env2 env3" with AB_ENV2 / AB_ENV3: more env legs against the current library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_ab}
mkdir -p $OUT
export PYTHONPATH=$R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 200 --timeout-method thread -s ${TESTK:+-k "$TESTK"} > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
if [ -n "$WINO" ]; then
  for lib in prev cur; do
    if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
    timeout -k 10 300 python -u tools/bench_wino3.py --quick > $OUT/wino3_$lib.log 2>&1 || { tail -5 $OUT/wino3_$lib.log; exit 3; }
    echo "$lib wino3 $(grep 'step totals' $OUT/wino3_$lib.log)"
  done
  unset TSPLAT_LIB
fi
for i in 1 2; do
  for leg in ${LEGS:-prev cur env}; do
    unset TSPLAT_LIB
    envs=""
    [ $leg = prev ] && export TSPLAT_LIB=tools/_bin/prev.so
    [ $leg = env ] && envs="$AB_ENV"
    [ $leg = env2 ] && envs="$AB_ENV2"
    [ $leg = env3 ] && envs="$AB_ENV3"
    [ $leg = env ] && [ -z "$AB_ENV" ] && continue
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench_${leg}_$i.log 2>&1 || { tail -5 $OUT/bench_${leg}_$i.log; exit 4; }
    echo "$leg $i c2 $(tail -1 $OUT/bench_${leg}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["frac"],4), d["roofline"]["avg_launch_ms"], round(d["roofline_step_dominant"]["ms_per_step"],3))')"
  done
done
