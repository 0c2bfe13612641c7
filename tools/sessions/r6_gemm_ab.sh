#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
for v in "" tools/var/gemm_v1.so tools/var/gemm_sb.so; do
  echo "== lib ${v:-default}"
  TSPLAT_LIB=$v timeout -k 10 120 python -u tools/bench_gemm_x3.py 2>&1 | grep -v amdgpu.ids || exit 1
done
