#!/bin/bash
# Kernels per stage segment of the replayed C2 step: rocprofv3 kernel trace of tools/graph_stages.py
# (stage-mark stamp kernels in the trace), digested on the box by tools/stage_kernels.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_stagek}
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/stk -o run -- python3 $R/tools/graph_stages.py --replays 3 > $OUT/stages.log 2>&1 || { tail -5 $OUT/stages.log; exit 1; }
cd $R
DB=$(find /tmp/stk -name "*.db" | head -1)
python3 tools/stage_kernels.py $DB --marks-per-step ${MARKS:-34} --top ${TOP:-8} > $OUT/stage_kernels.txt 2>&1 || { tail -5 $OUT/stage_kernels.txt; exit 2; }
grep -v amdgpu $OUT/stages.log | head -30
cat $OUT/stage_kernels.txt
