set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest tests/test_encoder_ops.py tests/test_modules.py -m gpu -v --timeout 120 --timeout-method thread -k "window_attention or x3 or uv_coarse or mvt" -s -rA > gpurun_out/r6e/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/bench_winattn.py --dtype bf16 --batch 16 > gpurun_out/r6e/wa.log 2>&1 && \
TSPLAT_WINATTN_V3_ROWS=0 timeout -k 10 120 python tools/bench_winattn.py --dtype bf16 --batch 16 >> gpurun_out/r6e/wa.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype bf16 --batch 16 --shift 0 >> gpurun_out/r6e/wa.log 2>&1 && \
TSPLAT_WINATTN_V3_ROWS=0 timeout -k 10 120 python tools/bench_winattn.py --dtype bf16 --batch 16 --shift 0 >> gpurun_out/r6e/wa.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6e/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6e/wa.log 2>&1
