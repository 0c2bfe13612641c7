#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 200 python -u tools/enc_graph_race.py 12 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/graph_vs_eager.py bf16x3 12 2>&1 | grep -v amdgpu.ids | tail -3; }
r camhoist0 TSPLAT_CAM_HOIST=0 && r camhoist0b TSPLAT_CAM_HOIST=0 && r dpbegin0 TSPLAT_DP_BEGIN_SIDE=0
for i in 1 2; do
for v in "" TSPLAT_CAM_HOIST=0 TSPLAT_DP_BEGIN_SIDE=0; do echo "bench ${v:-default} $(env $v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-140)"; done
done
