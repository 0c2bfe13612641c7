#!/bin/bash
# Same-box A/B of the direct-conv launch caps at batch 8 (C3 bf16 and fp32): old caps vs defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
O=gpurun_out/ab; mkdir -p $O
OLD="TSPLAT_CONV1_WAVES=4096 TSPLAT_CONV1_PAIRS=16 TSPLAT_CONV3_WAVES=4096"
NEW="TSPLAT_CONV_AB=new"
for r in 1 2; do
  for cfg in "$OLD" "$NEW"; do
    env $cfg timeout -k 10 300 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
    echo "c3 $cfg $(tail -1 $O/c3.log | grep -o '"value": [0-9.]*')"
  done
done
for cfg in "$OLD" "$NEW"; do
  env $cfg timeout -k 10 300 python bench.py --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > $O/b8.log 2>&1 || { tail -20 $O/b8.log; exit 1; }
  echo "b8 $cfg $(tail -1 $O/b8.log | grep -o '"value": [0-9.]*')"
done
