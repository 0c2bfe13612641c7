#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/graph_vs_eager.py bf16x3 8 2>&1 | grep -v amdgpu.ids | tail -5; }
r default "" && r zsplit0 TSPLAT_CONV_ZSPLIT=0 && r dpbegin0 TSPLAT_DP_BEGIN_SIDE=0 && r camhoist0 TSPLAT_CAM_HOIST=0 && r serial TSPLAT_STREAMS=0
