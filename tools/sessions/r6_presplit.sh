#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_conv.py tests/test_modules.py tests/test_e2e.py -m gpu -q --timeout 200 --timeout-method thread -s -k "gemm_x3 or depth_anything or graph_replays or bf16x3_step_vs" 2>&1 | grep -E "passed|failed|FAILED|golden.*depth_anything|replays vs" | tail -8
for i in 1 2; do for v in "X=0" "TSPLAT_MHA_PRESPLIT=0"; do echo "$v $(env $v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-120)"; done; done
