export PYTHONPATH=$PWD
O=gpurun_out/raster; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_raster.py -m gpu > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_raster.py --diag 0,2 || exit 1
