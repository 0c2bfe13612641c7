export PYTHONPATH=$PWD
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/on.log 2>&1 || exit 1
TSPLAT_CONV=off timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/off.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/on2.log 2>&1 || exit 1
for f in on off on2; do echo $f $(tail -1 $O/$f.log | cut -c80-140); done
