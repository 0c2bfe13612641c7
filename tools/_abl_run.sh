cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 300 python -m pytest tests/test_encoder_ops.py -q -m gpu -k "window" > gpurun_out/t_wa.log 2>&1; tail -1 gpurun_out/t_wa.log
for n in ${ABLS:-0}; do
  echo "ABL $n"
  TSPLAT_LIB=build/abl/lib$n.so TSPLAT_WINATTN=pair TSPLAT_WINATTN_KSPLIT=2 timeout -k 10 60 python tools/bench_winattn.py --batch 16 --iters 30 || exit 1
  TSPLAT_LIB=build/abl/lib$n.so timeout -k 10 60 python tools/bench_winattn.py --batch 2 --iters 50 || exit 1
done
