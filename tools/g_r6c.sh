set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops.py -m gpu -v --timeout 120 --timeout-method thread -k "uv_coarse" -s -rA > gpurun_out/r6c/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/bench_corr.py > gpurun_out/r6c/corr.log 2>&1 && \
TSPLAT_UV_COARSE_BITMAP=1 timeout -k 10 120 python tools/bench_corr.py >> gpurun_out/r6c/corr.log 2>&1 && \
timeout -k 10 120 python tools/bench_corr.py --batch 4 >> gpurun_out/r6c/corr.log 2>&1 && \
TSPLAT_UV_COARSE_BITMAP=1 timeout -k 10 120 python tools/bench_corr.py --batch 4 >> gpurun_out/r6c/corr.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 > gpurun_out/r6c/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6c/wa.log 2>&1 && \
TSPLAT_WINATTN_KSPLIT=2 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6c/wa.log 2>&1 && \
TSPLAT_WINATTN_KSPLIT=8 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6c/wa.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 --batch 16 >> gpurun_out/r6c/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 --batch 16 >> gpurun_out/r6c/wa.log 2>&1
