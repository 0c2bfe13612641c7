cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py -q -m gpu -k "window" > gpurun_out/wa_test.log 2>&1; tail -2 gpurun_out/wa_test.log
B="python tools/bench_winattn.py --dtype bf16"
for a in "" "--batch 16" "--batch 16 --shift 0"; do timeout -k 10 120 $B $a || exit 1; done
