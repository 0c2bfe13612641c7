#!/bin/bash
# Rasterizer block-relative power form: parity tests, raster-only and C2 A/B, raster kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-raster_rel}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests/test_raster.py tests/test_reference_golden.py -m gpu -x -q -s --timeout 300 > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep -i "flagged\|L-inf\|linf" $OUT/pytest.log | head -12
run() {
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py $extra --steps 20 --warmup 3 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:10.1f} {d['unit']} {d['ms_per_step']:8.4f} ms")
PY
}
run raster_rel "--workload raster"
run raster_plain "--workload raster" TSPLAT_RASTER_REL=0
run raster_rel2 "--workload raster"
run raster_plain2 "--workload raster" TSPLAT_RASTER_REL=0
run c2_rel ""
run c2_plain "" TSPLAT_RASTER_REL=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rel -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_rel.log 2>&1 || { echo prof failed; exit 1; }
grep -i "render\|preprocess" $OUT/prof_rel/run_kernel_stats.csv | cut -c1-160
echo done
