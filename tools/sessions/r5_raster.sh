#!/bin/bash
# Round-5 rasterizer probe: phase times with the render diagnostics (0 full, 2 key load + sort,
# 4 fetch + cull + compaction without blending), the per-wave distribution, and the raster bench line
# (HBM roofline of the whole call + the render kernel's VALU roofline).
# usage: TAG=<tag> [TESTS="tests/test_raster.py"] bash tools/sessions/r5_raster.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_raster}
mkdir -p $OUT
export PYTHONPATH=$R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 200 --timeout-method thread -s ${TESTK:+-k "$TESTK"} > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for lib in ${LIBS:-cur}; do
  unset TSPLAT_LIB
  [ $lib = prev ] && export TSPLAT_LIB=tools/_bin/prev.so
  timeout -k 10 300 python -u tools/bench_raster.py --diag ${DIAG:-0,2,4} --waves > $OUT/phases_$lib.log 2>&1 || { tail -5 $OUT/phases_$lib.log; exit 3; }
  cat $OUT/phases_$lib.log
  timeout -k 10 300 python -u bench.py --workload raster --no-cpu-baseline > $OUT/bench_raster_$lib.log 2>&1 || { tail -5 $OUT/bench_raster_$lib.log; exit 4; }
  tail -1 $OUT/bench_raster_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; v=d["roofline_render_valu"]; print("'$lib'", round(d["value"]), "views/s raster", round(r["avg_launch_ms"]*1e3,1), "us frac", round(r["frac"],3), "| render", round(v["avg_launch_ms"]*1e3,1), "us valu frac", round(v["frac"],3), "evals", v["entry_pixel_evals_per_launch"], "chunks", v["chunks_per_launch"], v["wave_cycles_p50_max"])'
done
