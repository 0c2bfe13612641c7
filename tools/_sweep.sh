cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py tests/test_modules.py -q -m gpu -k "window or mvt or backbone" > gpurun_out/wa_test.log 2>&1; tail -2 gpurun_out/wa_test.log
B="python tools/bench_winattn.py"
for a in "" "--shift 0" "--batch 16"; do timeout -k 10 120 $B $a || exit 1; done
timeout -k 10 120 env TSPLAT_WINATTN=pair $B --batch 16 || exit 1
timeout -k 10 120 env TSPLAT_WINATTN=32 $B || exit 1
