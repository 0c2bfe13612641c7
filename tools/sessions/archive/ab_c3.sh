#!/bin/bash
# C3 (batch 8, bf16 dense) A/B of the bf16-I/O norm kernels + their tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab_c3}
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_encoder_ops.py tests/test_e2e.py tests/test_modules.py -m gpu -x -q -s --timeout 300 \
    -k "group_norm or residual_ln or c3 or bf16 or depth_anything" > $OUT/pytest.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest.log; exit 1; }
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
run c3_old TSPLAT_BF16_NORMS=0
run c3_new2

rraster() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload raster --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']*1e3:7.1f} us/call  frac {d['roofline']['frac']:.3f}")
PY
}
timeout -k 10 300 python -u -m pytest tests/test_raster.py -m gpu -x -q --timeout 200 > $OUT/pytest_raster.log 2>&1 || { echo raster tests failed; tail -20 $OUT/pytest_raster.log; exit 1; }
tail -1 $OUT/pytest_raster.log
rraster rot_on
rraster rot_off TSPLAT_RASTER_ROT=0
rraster rot_on2
echo done2
