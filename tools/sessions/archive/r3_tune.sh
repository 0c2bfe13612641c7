#!/bin/bash
# Library GEMM re-tuning: fp32 (TunableOp, numerical check on) then bf16 (allow-list of hipBLASLt's
# heuristic top-k, every candidate logged before it runs); the new CSV is copied to gpurun_out; then
# the tuned-GEMM parity test and C2 / C3 with and without the file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-tune}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 500 python -u tools/tune_gemms.py > $OUT/tune_fp32.log 2>&1 || { echo "fp32 tune failed"; tail -20 $OUT/tune_fp32.log; exit 1; }
tail -3 $OUT/tune_fp32.log
timeout -k 10 600 python -u tools/tune_gemms_bf16.py > $OUT/tune_bf16.log 2>&1 || { echo "bf16 tune failed"; tail -20 $OUT/tune_bf16.log; exit 1; }
grep -v "^gemm_probe: candidate" $OUT/tune_bf16.log | grep -v amdgpu.ids | tail -30
cp transplat_amd/tuned/gemms_gfx950.csv $OUT/gemms_gfx950.csv
timeout -k 10 400 python -u -m pytest tests/test_e2e.py -m gpu -x -q --timeout 380 -k "tuned or c3" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
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
run c2_tuned ""
run c2_untuned "" TSPLAT_TUNED_GEMMS=0
run c3_tuned "$C3"
run c3_untuned "$C3" TSPLAT_TUNED_GEMMS=0
echo done
