#!/bin/bash
# DPT branch hoisting: the graph test with Depth-Anything on the current stream (backbone forked),
# then minimal nested-fork captures (each step only if the previous one ended cleanly).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/hoist_dbg2
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_e2e.py -m gpu -x -q --timeout 280 -k "graph_matches_eager" > $OUT/graph_hoist.log 2>&1 || { echo "graph hoist failed"; tail -5 $OUT/graph_hoist.log; exit 1; }
tail -1 $OUT/graph_hoist.log
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -q --timeout 280 -k "bf16" > $OUT/conv_bf16.log 2>&1 || { echo "conv bf16 failed"; tail -25 $OUT/conv_bf16.log; exit 1; }
tail -1 $OUT/conv_bf16.log
for m in flat nested_once nested; do
  timeout -k 10 120 python tools/graph_fork_repro.py $m > $OUT/repro_$m.log 2>&1 || { echo "repro $m failed rc=$?"; tail -3 $OUT/repro_$m.log; exit 1; }
  tail -1 $OUT/repro_$m.log
done
echo done
