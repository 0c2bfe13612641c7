#!/bin/bash
# SQ counters of the bf16 implicit-GEMM convolution (register-blocked form, 16 x 128 -> 128 at 64^2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
timeout -k 10 60 python tools/one_convbf16.py --iters 3 || exit 1
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM;SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/pmc_kernel.sh conv_bf16_kernel python3 $(pwd)/tools/one_convbf16.py --iters 5 > gpurun_out/pmc_convbf16.txt 2>&1; rc=$?
cat gpurun_out/pmc_convbf16.txt | tail -30; exit $rc
