cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py -q -m gpu -k window > gpurun_out/wa_test.log 2>&1; tail -2 gpurun_out/wa_test.log
B="python tools/bench_winattn.py"
for a in "" "--shift 0" "--batch 16" "--dtype bf16" "--dtype bf16 --batch 16"; do timeout -k 10 120 $B $a || exit 1; done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 200 rocprofv3 --pmc $C -d $GRAFT_REPO_ROOT/gpurun_out/wa_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_winattn.py --iters 5 > /dev/null 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wa_prof3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_winattn.py > /dev/null 2>&1 || exit 1
