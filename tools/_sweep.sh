cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py -q -m gpu -k "window" > gpurun_out/wa_test.log 2>&1; tail -3 gpurun_out/wa_test.log
B="python tools/bench_winattn.py"
timeout -k 10 120 $B --dtype bf16 || exit 1
timeout -k 10 120 $B --dtype bf16 --batch 16 || exit 1
timeout -k 10 120 $B --batch 16 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch 8 --dense-dtype bf16 --dominant win_attn --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; tail -1 gpurun_out/bench_c3.log | cut -c1-400
