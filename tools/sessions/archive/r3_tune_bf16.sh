#!/bin/bash
# bf16 library-GEMM tuning over hipBLASLt's heuristic top-k (tools/tune_gemms_bf16.py: each candidate's
# solution index is logged before it runs), then the tuned-GEMM parity tests and C3 with / without the
# recorded solutions. Needs tools/_bin/libgemm_probe.so (built on the CPU side, see gemm_probe.cpp).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-tune_bf16}
mkdir -p $OUT
export PYTHONPATH=$R
cp transplat_amd/tuned/gemms_gfx950.csv $OUT/gemms_before.csv
timeout -k 10 600 python -u tools/tune_gemms_bf16.py > $OUT/tune_bf16.log 2>&1 || { echo "bf16 tune failed"; tail -20 $OUT/tune_bf16.log; exit 1; }
grep -v "^gemm_probe: candidate" $OUT/tune_bf16.log | grep -v amdgpu.ids | tail -40
cp transplat_amd/tuned/gemms_gfx950.csv $OUT/gemms_gfx950.csv
timeout -k 10 400 python -u -m pytest tests/test_e2e.py -m gpu -x -q --timeout 380 -k "tuned or c3" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms")
PY
}
run c3_tuned
run c3_untuned TSPLAT_TUNED_GEMMS=0
run c3_tuned2
run c3_untuned2 TSPLAT_TUNED_GEMMS=0
echo done
