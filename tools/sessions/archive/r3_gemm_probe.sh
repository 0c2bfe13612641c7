#!/bin/bash
# bf16 GEMM allow-list tuning (dry run: probe + report) and the C3 im2col convolution candidates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-gemm_probe}
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 200 python tools/bench_conv_misc.py > $OUT/conv_misc.log 2>&1 || { echo "conv misc failed"; tail -5 $OUT/conv_misc.log; exit 1; }
grep -v amdgpu.ids $OUT/conv_misc.log
timeout -k 10 600 python -u tools/tune_gemms_bf16.py --dry > $OUT/tune_dry.log 2>&1 || { echo "tune failed"; tail -20 $OUT/tune_dry.log; exit 1; }
grep -v amdgpu.ids $OUT/tune_dry.log | grep -v "^gemm_probe: candidate" | tail -60
echo done
