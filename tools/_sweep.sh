cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py tests/test_modules.py -q -m gpu > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
for dom in uv_cross_table win_attn; do
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --dominant $dom --no-cpu-baseline > gpurun_out/b_$dom.log 2>&1 || { tail -5 gpurun_out/b_$dom.log; exit 1; }
tail -1 gpurun_out/b_$dom.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "views/s", round(d["ms_per_step"],2), "ms", d["roofline"])'
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1o -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_r1o.log 2>&1 || exit 1
