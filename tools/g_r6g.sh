set -o pipefail
mkdir -p gpurun_out/r6g
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops.py -m gpu -v --timeout 120 --timeout-method thread -k "x3_variants" -s -rA > gpurun_out/r6g/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6g/wa.log 2>&1 && \
TSPLAT_WINATTN_X3_XCD=window timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6g/wa.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/r6g/pmc_d_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $R/gpurun_out/r6g/pmc_d_$C.log 2>&1 || exit 1
  TSPLAT_WINATTN_X3_XCD=window timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/r6g/pmc_w_$C -o run --output-format csv -- python3 $R/tools/bench_winattn.py --batch 2 --dtype x3 --iters 20 > $R/gpurun_out/r6g/pmc_w_$C.log 2>&1 || exit 1
done
cd $R
f() { find gpurun_out/r6g/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/pmc_traffic.py $(f pmc_d_FETCH_SIZE) $(f pmc_d_WRITE_SIZE) win_attn_x3 gpurun_out/r6g/traffic_default.json
python3 tools/pmc_traffic.py $(f pmc_w_FETCH_SIZE) $(f pmc_w_WRITE_SIZE) win_attn_x3 gpurun_out/r6g/traffic_window.json
rm -rf gpurun_out/r6g/pmc_*_SIZE
