#!/bin/bash
# Round 4: auto form check after the staging rework, C2 A/B (fp32 vs bf16x3), per-op glue census of
# the bf16x3 step, rocprofv3 kernel trace of the bf16x3 C2 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g10}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > $OUT/pytest_w3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_w3.log | head; tail -3 $OUT/pytest_w3.log; exit 1; }
tail -1 $OUT/pytest_w3.log
timeout -k 10 200 python -u tools/bench_wino3.py --quick > $OUT/bench_wino3_auto.log 2>&1 || { tail -3 $OUT/bench_wino3_auto.log; exit 2; }
tail -1 $OUT/bench_wino3_auto.log
for d in bf16x3 fp32 bf16x3; do
  timeout -k 10 300 python -u bench.py --dense-dtype $d --no-cpu-baseline > $OUT/bench_c2_$d.log 2>&1 || { tail -5 $OUT/bench_c2_$d.log; exit 3; }
  echo "$d $(tail -1 $OUT/bench_c2_$d.log | cut -c1-140)"
done
timeout -k 10 300 python -u tools/op_stacks.py 1 bf16x3 > $OUT/op_stacks_x3.txt 2>&1 || { tail -5 $OUT/op_stacks_x3.txt; exit 4; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_x3 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c2_x3.log 2>&1 || exit 5
cd $R
python3 tools/prof_steps.py $OUT/prof_c2_x3/run_kernel_trace.csv > $OUT/c2_x3_per_step.txt 2>&1 || true
head -30 $OUT/c2_x3_per_step.txt | cut -c1-150
TSPLAT_LIB=tools/_bin/w3stamp.so timeout -k 10 120 python -u tools/w3_stamps.py > $OUT/w3_stamps.log 2>&1 || { tail -5 $OUT/w3_stamps.log; exit 6; }
grep -v amdgpu $OUT/w3_stamps.log
for m in plain xf32 tf32; do
  case $m in
    plain) timeout -k 10 120 python -u tools/bench_xf32.py > $OUT/xf32_$m.log 2>&1 ;;
    xf32) HIPBLASLT_OVERRIDE_COMPUTE_TYPE_XF32=1 timeout -k 10 120 python -u tools/bench_xf32.py > $OUT/xf32_$m.log 2>&1 ;;
    tf32) timeout -k 10 120 python -u tools/bench_xf32.py --allow-tf32 > $OUT/xf32_$m.log 2>&1 ;;
  esac || { tail -5 $OUT/xf32_$m.log; exit 7; }
  grep -v amdgpu $OUT/xf32_$m.log
done
