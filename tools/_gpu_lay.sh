export PYTHONPATH=$PWD
O=gpurun_out/lay; mkdir -p $O
timeout -k 10 500 python tools/conv_layout_ab.py > $O/conv_ab.txt 2>&1 || exit 1
