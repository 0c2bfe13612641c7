#!/bin/bash
# C3: split-bf16 correlation table + NCHW resize; tests, A/B, profile with MIOpen's search on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-ab_c3b}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest tests/test_encoder_ops.py tests/test_e2e.py tests/test_modules.py -m gpu -x -q -s --timeout 300 \
    -k "uv_cross or c3 or depth_anything or bf16" > $OUT/pytest.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep "C3 bf16" $OUT/pytest.log | cut -c1-200
run() {
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms  attn {d['roofline']['frac']:.3f}")
PY
}
run c3_new
run c3_notable TSPLAT_UV_TABLE_BF16=0
run c3_new2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.log 2>&1 || { echo prof c3 failed; exit 1; }
echo done
