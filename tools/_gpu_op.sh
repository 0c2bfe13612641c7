R=$(pwd); OUT=$R/gpurun_out/op; mkdir -p $OUT; export PYTHONPATH=$R
timeout -k 10 600 python tools/op_profile.py > $OUT/op.txt 2>&1 || exit 1
