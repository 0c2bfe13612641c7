#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_conv.py tests/test_modules.py -m gpu -q --timeout 200 --timeout-method thread -k "residual_ln or depth_anything or dinov2" 2>&1 | grep -E "passed|failed|FAILED" | tail -3
for i in 1 2 3; do for v in "" tools/var/rln_prev.so; do echo "bench ${v:-hoisted} $(TSPLAT_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c80-120)"; done; done
