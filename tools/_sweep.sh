cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py -q -m gpu -k "window" > gpurun_out/wa_test.log 2>&1; tail -2 gpurun_out/wa_test.log
B="python tools/bench_winattn.py"
for a in "" "--batch 16" "--dtype bf16" "--dtype bf16 --batch 16"; do timeout -k 10 120 $B $a || exit 1; done
