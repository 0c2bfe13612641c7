#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/step_err_ab.py "$1" $3 2>&1 | grep -v amdgpu.ids | tail -1; }
r tuned "" --tuned && r tuned_x3v1 TSPLAT_WINATTN_X3=v1 --tuned && r tuned_few0 TSPLAT_CONV_FEW=0 --tuned && r tuned_attnoff TSPLAT_ATTN_X3=0 --tuned
