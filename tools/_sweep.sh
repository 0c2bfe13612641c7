cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
B="python tools/bench_winattn.py"
timeout -k 10 200 python -m pytest tests/test_encoder_ops.py -q -m gpu -k window > gpurun_out/wa_test.log 2>&1; tail -2 gpurun_out/wa_test.log
for cfg in "TSPLAT_WINATTN=32" "TSPLAT_WINATTN=32 TSPLAT_WINATTN_KSPLIT=4"; do
  timeout -k 10 120 env $cfg $B || exit 1
done
timeout -k 10 120 env TSPLAT_WINATTN=32 $B --batch 16 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wa_prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_winattn.py > $GRAFT_REPO_ROOT/gpurun_out/wa_prof.log 2>&1 || exit 1
