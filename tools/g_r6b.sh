set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r6b/bench_c2.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 > gpurun_out/r6b/wa_x3.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype bf16 --batch 16 > gpurun_out/r6b/wa_bf16_b16.log 2>&1 && \
timeout -k 10 120 python tools/bench_corr.py > gpurun_out/r6b/corr.log 2>&1
