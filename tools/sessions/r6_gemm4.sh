#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -q --timeout 200 --timeout-method thread -s -k "gemm_x3" 2>&1 | grep -E "passed|failed|Error" | tail -3
for v in "" tools/var/gemm_nmajor.so "" tools/var/gemm_nmajor.so; do echo "== ${v:-kmajor}"; TSPLAT_LIB=$v timeout -k 10 120 python -u tools/bench_gemm_x3.py 2>&1 | grep -v amdgpu.ids; done
