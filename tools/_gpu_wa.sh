export PYTHONPATH=$PWD
O=gpurun_out/wa; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encoder_ops.py -m gpu -k "window_attention" > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
for v in quad 32; do TSPLAT_WINATTN=$v timeout -k 10 60 python tools/bench_winattn.py --batch 2 --iters 100 || exit 1; done
timeout -k 10 60 python tools/bench_winattn.py --batch 2 --iters 100 --shift 0 || exit 1
timeout -k 10 60 python tools/bench_winattn.py --batch 4 --iters 50 || exit 1
TSPLAT_WINATTN=32 timeout -k 10 60 python tools/bench_winattn.py --batch 4 --iters 50 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_e2e.py -m gpu -k precast > $O/test_e2e.log 2>&1; tail -3 $O/test_e2e.log
