set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r4
rm -f gpurun_out/r4/w3abl.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > gpurun_out/r4/pytest_w3.log 2>&1 || exit 1
TSPLAT_WINO3_STAGE=1 timeout -k 10 120 python -u tools/ab_w3.py 1 2 3 4 >> gpurun_out/r4/w3abl.log 2>&1 || exit 2
for lib in "" tools/_bin/w3abl1.so tools/_bin/w3abl2.so tools/_bin/w3abl3.so; do
  TSPLAT_WINO3_STAGE=0 TSPLAT_LIB=$lib timeout -k 10 120 python -u tools/ab_w3.py 1 2 4 >> gpurun_out/r4/w3abl.log 2>&1 || exit 3
done
