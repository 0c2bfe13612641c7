#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_encoder_ops.py tests/test_modules.py tests/test_e2e.py tests/test_reference_golden.py -m gpu -q --timeout 300 --timeout-method thread -s -k "uv_cross or depth_predictor or encoder or graph_replays or bf16x3_step_vs" 2>&1 | grep -E "passed|failed|FAILED|golden.*bf16x3|replays vs|bf16x3 vs fp32" | grep -v "^ " | tail -16
for i in 1 2 3; do for v in "X=0" "TSPLAT_UV_TABLE_GEMM_X3=0"; do echo "$v $(env $v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-120)"; done; done
