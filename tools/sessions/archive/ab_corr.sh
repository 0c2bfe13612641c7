cd $GRAFT_REPO_ROOT && export PYTHONPATH=.
timeout -k 10 120 python -m pytest tests/test_encoder_ops.py -m gpu -q -x --timeout 60 -k "coarse" 2>&1 | tail -2 || exit 1
for r in 1 2; do for lib in tools/_bin/libtransplat_base.so transplat_amd/libtransplat_hip.so; do for d in 1 2 3 0; do
  TSPLAT_LIB=$lib TSPLAT_CORR_DIAG=$d timeout -k 10 60 python tools/bench_corr.py --iters 200 2>&1 | grep uv_coarse | sed "s#^#$(basename $lib) diag=$d #" || exit 1
done; done; done
