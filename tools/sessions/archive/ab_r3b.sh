#!/bin/bash
# Raster preprocess A/B (views per workgroup) + raster tests; C3 op call sites and kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$(pwd)/gpurun_out/${TAG:-ab_r3b}
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_raster.py tests/test_reference_golden.py -m gpu -x -q --timeout 200 > $OUT/pytest_raster.log 2>&1 || { echo raster tests failed; tail -20 $OUT/pytest_raster.log; exit 1; }
tail -1 $OUT/pytest_raster.log
rraster() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload raster --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']*1e3:7.1f} us/call  frac {d['roofline']['frac']:.3f}")
PY
}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_raster -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload raster --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_raster.log 2>&1 || { echo prof failed; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/op_stacks.py 8 bf16 > $OUT/ops_c3.log 2>&1 || { tail -5 $OUT/ops_c3.log; exit 1; }
head -30 $OUT/ops_c3.log
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3.log 2>&1 || { echo prof c3 failed; exit 1; }
echo done
