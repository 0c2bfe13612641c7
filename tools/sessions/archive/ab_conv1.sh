#!/bin/bash
# Same-box A/B of the direct kernel's 1x1 launch shape (TSPLAT_CONV1_WAVES / TSPLAT_CONV1_PAIRS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
O=gpurun_out/ab; mkdir -p $O
TSPLAT_CONV1_WAVES=16384 TSPLAT_CONV1_PAIRS=8 timeout -k 10 300 python -u -m pytest tests/test_conv.py tests/test_modules.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  for cfg in "TSPLAT_CONV1_WAVES=4096 TSPLAT_CONV1_PAIRS=16" "TSPLAT_CONV1_WAVES=16384 TSPLAT_CONV1_PAIRS=8" "TSPLAT_CONV1_WAVES=8192 TSPLAT_CONV1_PAIRS=16" "TSPLAT_CONV1_WAVES=16384 TSPLAT_CONV1_PAIRS=4"; do
    env $cfg timeout -k 10 300 $B > $O/e2e.log 2>&1 || { tail -20 $O/e2e.log; exit 1; }
    echo "$cfg $(tail -1 $O/e2e.log | grep -o '"value": [0-9.]*')"
  done
done
