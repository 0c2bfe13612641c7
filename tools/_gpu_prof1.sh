R=$(pwd); OUT=$R/gpurun_out/p1; mkdir -p $OUT; export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
cd $R && python tools/prof_steps.py $(find $OUT/prof -name '*kernel_trace.csv' | head -1) --top 70 > $OUT/per_step.txt && find $OUT/prof -name '*.csv' -delete
