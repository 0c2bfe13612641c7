#!/bin/bash
# g33: coarse correlation with 8 workgroups per CU (corners recomputed instead of held, 64 VGPRs) vs the
# previous library (tools/_bin/prev.so): coarse tests, microbenchmark, C2, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g33
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_encoder_ops.py \
  -k "uv_coarse" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
    timeout -k 10 120 python -u tools/bench_corr.py > $OUT/corr.log 2>&1 || { tail -3 $OUT/corr.log; exit 3; }
    echo "$lib $i: $(grep -v amdgpu $OUT/corr.log | tail -1 | cut -c1-150)"
  done
done
for i in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_${lib}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${lib}_$i.log; exit 4; }
    echo "$lib $i c2 $(tail -1 $OUT/bench_c2_${lib}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')"
  done
done
