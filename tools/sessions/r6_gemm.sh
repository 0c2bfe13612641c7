#!/bin/bash
# hand-written bf16x3 GEMM: tests, microbench vs hipBLASLt, C2 A/B (TSPLAT_GEMM_X3=0 / 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/r6_gemm; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv.py tests/test_e2e.py tests/test_reference_golden.py tests/test_modules.py -m gpu -v --timeout 200 --timeout-method thread -s -k "gemm_x3 or residual_ln_slabs or graph_replays or bf16x3_step_vs or depth_anything or dinov2" > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|rel err|replays vs|bf16x3 vs fp32" $OUT/pytest.log | grep -v "^tests.*PASSED" | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_dino_gemm.py > $OUT/gemm_bench.log 2>&1 || exit 1
grep -v amdgpu $OUT/gemm_bench.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1
TSPLAT_GEMM_X3=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_lib_$i.log 2>&1 || exit 1
done
for f in $OUT/bench_*.log; do echo $f $(tail -1 $f | cut -c1-140); done
