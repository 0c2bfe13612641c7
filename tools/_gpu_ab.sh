export PYTHONPATH=$PWD
mkdir -p gpurun_out/ab
for v in all dpt head none; do
TSPLAT_NO_CONV_EPI=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab/b_$v.log 2>&1 || exit 1
echo "no_conv_epi=$v $(tail -1 gpurun_out/ab/b_$v.log | cut -c90-150)"
done
