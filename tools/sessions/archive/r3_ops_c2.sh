#!/bin/bash
# Op call-site census of one eager C2 step (which Python lines launch PyTorch's own kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/${TAG:-ops_c2}
mkdir -p $OUT
timeout -k 10 300 python tools/op_stacks.py 1 fp32 > $OUT/ops_c2.log 2>&1 || { tail -5 $OUT/ops_c2.log; exit 1; }
head -70 $OUT/ops_c2.log
