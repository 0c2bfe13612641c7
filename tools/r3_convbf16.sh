#!/bin/bash
# bf16 implicit-GEMM conv: tests, per-shape timing vs MIOpen, workgroup-count A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-convbf16}
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -q --timeout 280 -k "bf16" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -25 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/bench_conv_bf16.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
grep -v amdgpu.ids $OUT/bench.log
for g in 4; do
  TSPLAT_CONVBF16_OCC=$g timeout -k 10 300 python tools/bench_conv_bf16.py > $OUT/bench_occ$g.log 2>&1 || { echo "occ $g failed"; exit 1; }
  echo "occ $g"; grep -v amdgpu.ids $OUT/bench_occ$g.log | tail -n +2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OLDPWD/$OUT/prof -o run --output-format csv -- python3 $OLDPWD/tools/bench_conv_bf16.py --iters 5 > $OLDPWD/$OUT/prof.log 2>&1 || { echo prof failed; exit 1; }
echo done
