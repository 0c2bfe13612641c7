export PYTHONPATH=$PWD
O=gpurun_out/ab; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 $B > $O/a1.log 2>&1 || exit 1
TSPLAT_UNET_GEMM1X1=0 timeout -k 10 300 $B > $O/b1.log 2>&1 || exit 1
timeout -k 10 300 $B > $O/a2.log 2>&1 || exit 1
TSPLAT_UNET_GEMM1X1=0 timeout -k 10 300 $B > $O/b2.log 2>&1 || exit 1
for f in a1 b1 a2 b2; do echo $f $(tail -1 $O/$f.log | cut -c80-140); done
