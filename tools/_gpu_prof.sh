R=$(pwd); OUT=$R/gpurun_out/final; mkdir -p $OUT; export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_fp32_b1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_e2e_fp32_b1.log 2>&1 || exit 1
echo e2e done
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 $R/bench.py --batch 8 --dense-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-conv-search > $OUT/prof_c3.log 2>&1 || exit 1
echo c3 done
