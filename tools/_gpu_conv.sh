export PYTHONPATH=$PWD
O=gpurun_out/conv; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -m gpu > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_conv.py > $O/bench.txt 2>&1 || exit 1
