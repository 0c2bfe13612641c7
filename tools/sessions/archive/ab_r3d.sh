#!/bin/bash
# C3 with the pipelined bf16 conv (occupancy 2 / 4) vs MIOpen; tests first; steady-state C3 profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-ab_r3d}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests/test_conv.py tests/test_e2e.py tests/test_modules.py -m gpu -x -q -s --timeout 300 \
    -k "bf16 or c3 or graph or unet or depth_predictor_gpu or depth_anything" > $OUT/pytest.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep "C3 bf16" $OUT/pytest.log | cut -c1-200
run() {
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py $extra --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms  attn {d['roofline']['frac']:.3f}")
PY
}
C3="--batch 8 --dense-dtype bf16"
run c3_conv "$C3"
run c3_conv_occ4 "$C3" TSPLAT_CONVBF16_OCC=4
run c3_noconv "$C3" TSPLAT_CONV_BF16=0
run c3_conv2 "$C3"
run c2 ""
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 12 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.log 2>&1 || { echo prof c3 failed; exit 1; }
python3 $R/tools/prof_steps.py $OUT/prof_c3/run_kernel_trace.csv > $OUT/c3_per_step.txt 2>&1 || true
cd $R && timeout -k 10 300 python tools/op_stacks.py 8 bf16 > $OUT/ops_c3.log 2>&1 || { echo ops failed; exit 1; }
echo done
