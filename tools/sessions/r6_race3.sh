#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/enc_graph_race.py 12 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200; }
r default "" && r bitmap TSPLAT_UV_COARSE_BITMAP=1 && r msdaraw0 TSPLAT_MSDA_RAW=0 && r wpe6 TSPLAT_CORR_RUN_WPE=6 && r dpbegin0 TSPLAT_DP_BEGIN_SIDE=0 && r default2 ""
