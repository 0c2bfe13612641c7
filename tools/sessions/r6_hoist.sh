#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
for i in 1 2 3; do for v in "X=0" "TSPLAT_DPT_HOIST=1"; do echo "$v $(env $v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-120)"; done; done
TSPLAT_DPT_HOIST=1 timeout -k 10 200 python -u tools/enc_graph_race.py 12 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-120
