#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/graph_vs_eager.py 2>&1 | grep -v amdgpu.ids | tail -5; }
r untuned TSPLAT_TUNED_GEMMS=0 && r untuned_b TSPLAT_TUNED_GEMMS=0 && r tuned_linx0 TSPLAT_LINX=0 && r tuned_again ""
