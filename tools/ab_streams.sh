#!/bin/bash
# A/B of the concurrent encoder branches and of the HIP runtime's graph-execution knobs, on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_streams
mkdir -p $OUT
export PYTHONPATH=$(pwd)
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:28s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms  attn {d['roofline']['frac']:.3f}")
PY
}
timeout -k 10 300 python -u -m pytest tests/test_raster.py -m gpu -x -q -s --timeout 200 > $OUT/pytest_raster.log 2>&1 || { echo raster tests failed; tail -20 $OUT/pytest_raster.log; exit 1; }
grep "raster parity" $OUT/pytest_raster.log | cut -c1-160
run streams_off TSPLAT_STREAMS=0
run streams_on TSPLAT_STREAMS=1
run on_nopacket TSPLAT_STREAMS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run off_nopacket TSPLAT_STREAMS=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run on_queues4 TSPLAT_STREAMS=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run on_queues2 TSPLAT_STREAMS=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
run streams_off2 TSPLAT_STREAMS=0
run streams_on2 TSPLAT_STREAMS=1
rraster() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload raster --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:28s} {d['value']:8.1f} views/s {d['ms_per_step']*1e3:7.1f} us/call  frac {d['roofline']['frac']:.3f}")
PY
}
rraster raster_sub1 TSPLAT_RASTER_SUB=1
rraster raster_sub0 TSPLAT_RASTER_SUB=0
rraster raster_sub1b TSPLAT_RASTER_SUB=1
