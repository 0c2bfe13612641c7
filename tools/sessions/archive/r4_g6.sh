#!/bin/bash
# Round 4: bf16x3 Winograd census of the C2 step, DPT NCHW A/B, SQ counters of the form-4 kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
OUT=gpurun_out/r4_g6
mkdir -p $OUT
timeout -k 10 200 python -u tools/wino_census.py bf16x3 > $OUT/wino_census_x3.log 2>&1 || { tail -5 $OUT/wino_census_x3.log; exit 1; }
cat $OUT/wino_census_x3.log | grep -v amdgpu
for i in 1 2; do
  for v in 0 1; do
    TSPLAT_DPT_NCHW3=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_nchw3_${v}_$i.log 2>&1 || exit 2
    echo "nchw3=$v $i $(tail -1 $OUT/bench_nchw3_${v}_$i.log | cut -c90-140)"
  done
done
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
  timeout -k 10 300 bash tools/pmc_kernel.sh "wino3" python3 $PWD/tools/one_wino3.py 2 163 168 256 256 > $OUT/pmc_form4.log 2>&1 || { tail -5 $OUT/pmc_form4.log; exit 3; }
cat $OUT/pmc_form4.log
