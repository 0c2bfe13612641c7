#!/bin/bash
# Round-3 A/B session: correctness of the changed kernels first (window attention x16 / x32,
# attention + merge, raster vs the literal oracle), then same-box A/Bs (e2e: streams, x16 attention;
# raster: 4x4 sub-block walk). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab_r3}
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_encoder_ops.py tests/test_raster.py -m gpu -x -q -s --timeout 200 \
    -k "window_attention_kernel or attention_merge or raster or uv_coarse" > $OUT/pytest.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep "raster parity (256\|raster parity (DTU" $OUT/pytest.log | cut -c1-200
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = d["roofline"]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms  attn {r['frac']:.3f} ({r['avg_launch_ms']*1e3:.1f} us)")
PY
}
rraster() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload raster --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']*1e3:7.1f} us/call  frac {d['roofline']['frac']:.3f}")
PY
}
for arg in ${AB_LIST:-corr e2e raster}; do
  if [ $arg = corr ]; then
    for G in 1 0 1; do
      TSPLAT_UV_COARSE_GROUP=$G timeout -k 10 120 python tools/bench_corr.py > $OUT/corr_g$G.log 2>&1 || { echo corr failed; tail -3 $OUT/corr_g$G.log; exit 1; }
      echo "uv_coarse group=$G: $(tail -1 $OUT/corr_g$G.log)"
    done
  fi
  if [ $arg = e2e ]; then
    run base
    run x32 TSPLAT_WA16=0
    run streams_off TSPLAT_STREAMS=0
    run nopacket DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
    run base2
  fi
  if [ $arg = raster ]; then
    rraster raster_sub1 TSPLAT_RASTER_SUB=1
    rraster raster_sub0 TSPLAT_RASTER_SUB=0
    rraster raster_sub1b TSPLAT_RASTER_SUB=1
  fi
done
echo done
