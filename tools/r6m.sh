export PYTHONPATH=$PWD
O=gpurun_out/r6_m; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_conv.py -k "few" -m gpu -q --timeout 120 --timeout-method thread > $O/few_tests.log 2>&1 || exit 1
timeout -k 10 100 python tools/fewch_conv.py > $O/fewch.log 2>&1 || exit 1
FORMS=4,6,7 timeout -k 10 100 python tools/wino3_forms.py "2,163,168,256,256" "2,168,84,256,256" "2,128,128,64,64" > $O/forms.log 2>&1
for i in 1 2; do
 TSPLAT_CONV_FEW=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2_off_$i.log 2>&1 || exit 1
 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2_on_$i.log 2>&1 || exit 1
done
