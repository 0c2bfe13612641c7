export PYTHONPATH=$PWD
O=gpurun_out/conv; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_ksplit_sweep.py > $O/ksweep.txt 2>&1 || exit 1
timeout -k 10 400 python tools/bench_conv.py > $O/bench.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b0.log 2>&1 || exit 1
tail -1 $O/b0.log | cut -c1-200
