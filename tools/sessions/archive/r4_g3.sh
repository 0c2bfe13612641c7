set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r4
rm -f gpurun_out/r4/w3abl.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > gpurun_out/r4/pytest_w3.log 2>&1 || exit 1
TSPLAT_WINO3_STAGE=1 timeout -k 10 120 python -u tools/ab_w3.py 1 2 3 4 >> gpurun_out/r4/w3abl.log 2>&1 || exit 2
for lib in "" tools/_bin/w3abl1.so tools/_bin/w3abl2.so tools/_bin/w3abl3.so; do
  TSPLAT_WINO3_STAGE=0 TSPLAT_LIB=$lib timeout -k 10 120 python -u tools/ab_w3.py 1 2 4 >> gpurun_out/r4/w3abl.log 2>&1 || exit 3
done
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_e2e.py tests/test_reference_golden.py tests/test_encoder_ops.py -k "bf16x3 or c3_stated or encoder_gpu or window_attention_kernel or attention_merge" -m gpu > gpurun_out/r4/pytest_e2e_x3.log 2>&1 || exit 4
timeout -k 10 240 python -u tools/bench_wino3.py --quick > gpurun_out/r4/bench_wino3_st.log 2>&1 || exit 5
timeout -k 10 200 python -u tools/bench_split_gemm.py > gpurun_out/r4/split_gemm2.log 2>&1 || exit 6
