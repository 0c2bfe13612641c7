#!/bin/bash
# Which round-6 change moved the bf16x3-vs-fp32 pixel mean (3.1e-5 -> 1.3e-4): the same measurement
# under each A/B knob.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r6_errab; mkdir -p $OUT
export PYTHONPATH=$(pwd)
r() { echo "== $1"; env $2 timeout -k 10 200 python -u tools/step_err_ab.py "$1" 2>&1 | grep -v amdgpu.ids | tail -1; }
r default "" && r few0 TSPLAT_CONV_FEW=0 && r x3v1 TSPLAT_WINATTN_X3=v1 && r bitmap TSPLAT_UV_COARSE_BITMAP=1 \
 && r libfree0 TSPLAT_CONV_LIBFREE_X3=0 && r attnx3off TSPLAT_ATTN_X3=0
