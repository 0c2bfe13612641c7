export PYTHONPATH=$PWD
O=gpurun_out/misc; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_raster.py -m gpu > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_raster.py --diag 0 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b0.log 2>&1 || exit 1
tail -1 $O/b0.log | cut -c1-240
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --conv-search > $O/b1.log 2>&1 || exit 1
tail -1 $O/b1.log | cut -c1-240
