#!/bin/bash
# g28: persistent bf16x3 Winograd with resident A fragments for two-chunk inputs (ci 17..32), auto-chosen
# for 32-channel big maps, vs the previous library (tools/_bin/prev.so = the commit before): conv tests,
# Winograd census (auto form), C2 alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g28
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv.py \
  -k "wino_bf16x3" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -2 $OUT/pytest.log
for lib in prev cur; do
  if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
  timeout -k 10 300 python -u tools/bench_wino3.py --quick > $OUT/wino3_$lib.log 2>&1 || { tail -5 $OUT/wino3_$lib.log; exit 3; }
  echo "== $lib"; grep -E "32, 256, 256|step totals" $OUT/wino3_$lib.log
done
for i in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_${lib}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${lib}_$i.log; exit 4; }
    echo "$lib $i c2 $(tail -1 $OUT/bench_c2_${lib}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')"
  done
done
