#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export PMC_GROUPS="FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
bash tools/pmc_kernel.sh gemm_x3_kernel python3 $R/tools/one_gemm.py 650 768 3072 1 gelu 20
