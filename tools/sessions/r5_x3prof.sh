#!/bin/bash
# bf16x3 attention diagnostics: per-workgroup phase clocks (stamp build), SQ counters, and the
# FETCH_SIZE / WRITE_SIZE traffic digest the bench line reads (profiles/<round>/traffic_win_attn_bf16x3_b1.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r5_x3prof}
mkdir -p $OUT
export PYTHONPATH=$R
TSPLAT_LIB=tools/_bin/wastamp.so timeout -k 10 120 python -u tools/wa_stamps.py --x3 > $OUT/stamps_x3.log 2>&1 || { tail -5 $OUT/stamps_x3.log; exit 1; }
grep -v amdgpu $OUT/stamps_x3.log
TSPLAT_LIB=tools/_bin/wastamp.so timeout -k 10 120 python -u tools/wa_stamps.py > $OUT/stamps_x32.log 2>&1 || { tail -5 $OUT/stamps_x32.log; exit 1; }
grep -v amdgpu $OUT/stamps_x32.log | head -4
timeout -k 10 400 bash tools/pmc_kernel.sh win_attn_x3 python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $OUT/sq_x3.txt 2>&1 || { tail -5 $OUT/sq_x3.txt; exit 1; }
cat $OUT/sq_x3.txt
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_x3_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $OUT/pmc_x3_$C.log 2>&1 || exit 1
done
cd $R
f() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/pmc_traffic.py $(f pmc_x3_FETCH_SIZE) $(f pmc_x3_WRITE_SIZE) win_attn_x3 $OUT/traffic_win_attn_bf16x3_b1.json && cat $OUT/traffic_win_attn_bf16x3_b1.json
