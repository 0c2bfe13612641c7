#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -q --timeout 200 --timeout-method thread -k "gemm_x3" 2>&1 | grep -E "passed|failed|FAILED" | tail -3
for v in "" tools/var/gemm_n2.so "" tools/var/gemm_n2.so; do echo "== ${v:-nset3}"; TSPLAT_LIB=$v timeout -k 10 120 python -u tools/bench_gemm_x3.py 2>&1 | grep -v amdgpu.ids; done
for i in 1 2; do for v in "" tools/var/gemm_n2.so; do echo "bench ${v:-nset3} $(TSPLAT_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-120)"; done; done
