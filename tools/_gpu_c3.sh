export PYTHONPATH=$PWD
mkdir -p gpurun_out/c3
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_e2e.py -m gpu -k precast > gpurun_out/c3/test.log 2>&1; rc=$?; tail -3 gpurun_out/c3/test.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3/bench.log 2>&1 || exit 1
tail -1 gpurun_out/c3/bench.log | cut -c1-250
