set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r4
timeout -k 10 240 python -u tools/bench_wino3.py > gpurun_out/r4/bench_wino3.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_encoder_ops.py tests/test_e2e.py -k "uv_cross or bf16x3 or c3_stated" -m gpu > gpurun_out/r4/pytest_e2e_x3.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --dense-dtype fp32 --no-cpu-baseline > gpurun_out/r4/bench_c2_fp32.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --dense-dtype bf16x3 --no-cpu-baseline > gpurun_out/r4/bench_c2_x3.log 2>&1 || exit 4
