set -o pipefail
mkdir -p gpurun_out/r6i
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops.py -m gpu -v --timeout 120 --timeout-method thread -k "uv_coarse" -s -rA > gpurun_out/r6i/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 120 python tools/bench_corr.py >> gpurun_out/r6i/corr.log 2>&1 && \
TSPLAT_CORR_RUN_WPE=6 timeout -k 10 120 python tools/bench_corr.py >> gpurun_out/r6i/corr.log 2>&1 && \
TSPLAT_UV_COARSE_BITMAP=1 timeout -k 10 120 python tools/bench_corr.py >> gpurun_out/r6i/corr.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/bench_corr.py --batch 4 >> gpurun_out/r6i/corr.log 2>&1 && \
TSPLAT_CORR_RUN_WPE=6 timeout -k 10 120 python tools/bench_corr.py --batch 4 >> gpurun_out/r6i/corr.log 2>&1
TSPLAT_LIB=tools/wastamp_tmp.so timeout -k 10 120 python tools/wa_stamps.py --bf16 > gpurun_out/r6i/stamps_v3.log 2>&1
