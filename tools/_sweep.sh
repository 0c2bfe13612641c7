cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/rr_pmc -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rr_pmc.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $R/gpurun_out/rr_pmc2 -o run --output-format csv -- python3 $R/bench.py --workload raster --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rr_pmc2.log 2>&1 || exit 1
