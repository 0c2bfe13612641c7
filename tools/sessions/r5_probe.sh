#!/bin/bash
# Round-5 probe: module-golden errors printed per dense mode (for the tightened bounds), the graph
# launch-cost probe, and the C2 step with the concurrent branches off (serial graph).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_probe}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_modules.py tests/test_reference_golden.py tests/test_capi.py -m gpu -s -q \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python tools/graph_launch_probe.py 660 50 > $OUT/graph_probe.log 2>&1 || exit 1
cat $OUT/graph_probe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.log 2>&1 || exit 1
TSPLAT_STREAMS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2_serial.log 2>&1 || exit 1
for f in bench_c2 bench_c2_serial; do tail -1 $OUT/$f.log | cut -c1-200; done
