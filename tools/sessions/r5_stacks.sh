#!/bin/bash
# Round-5 glue attribution: which call sites launch PyTorch kernels in one eager step (C2 and C3 as
# stated), tools/op_stacks.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_stacks}
mkdir -p $OUT
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python -u tools/op_stacks.py 8 bf16x3 bf16 > $OUT/stacks_c3.log 2>&1 || { tail -5 $OUT/stacks_c3.log; exit 1; }
timeout -k 10 200 python -u tools/op_stacks.py 1 bf16x3 > $OUT/stacks_c2.log 2>&1 || { tail -5 $OUT/stacks_c2.log; exit 1; }
head -60 $OUT/stacks_c3.log
