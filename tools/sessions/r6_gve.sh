#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/graph_vs_eager.py 2>&1 | grep -v amdgpu.ids | tail -5; }
r default "" && r serial TSPLAT_STREAMS=0 && r x3v1 TSPLAT_WINATTN_X3=v1 && r few0 TSPLAT_CONV_FEW=0
