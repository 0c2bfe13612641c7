set -o pipefail
mkdir -p gpurun_out/r6h
R=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_encoder_ops.py tests/test_modules.py -m gpu -v --timeout 120 --timeout-method thread -k "window_attention or x3 or mvt" -s -rA > gpurun_out/r6h/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TSPLAT_LIB=tools/wastamp_tmp.so timeout -k 10 120 python tools/wa_stamps.py --x3 > gpurun_out/r6h/stamps_v2.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6h/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6h/wa.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/r6h/pmc_d_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $R/gpurun_out/r6h/pmc_d_$C.log 2>&1 || exit 1
done
cd $R
f() { find gpurun_out/r6h/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/pmc_traffic.py $(f pmc_d_FETCH_SIZE) $(f pmc_d_WRITE_SIZE) win_attn_x3 gpurun_out/r6h/traffic_win_attn_bf16x3_b1.json
rm -rf gpurun_out/r6h/pmc_*_SIZE
