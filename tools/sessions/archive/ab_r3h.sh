#!/bin/bash
# bf16 convolution: the nearest-2x widening moved from the loads to the staging (conv tests, C3 A/B
# against the previous build in tools/_bin/libtransplat_base.so), then the full GPU suite + benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/${TAG:-r3h}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -q --timeout 200 --timeout-method thread -k bf16 > $OUT/pytest_conv.log 2>&1; rc=$?
tail -1 $OUT/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for lib in tools/_bin/libtransplat_base.so transplat_amd/libtransplat_hip.so; do
  TSPLAT_LIB=$lib timeout -k 10 300 python bench.py --batch 8 --dense-dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_$(basename $lib .so)_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3))" $OUT/c3_$(basename $lib .so)_$r.log
done; done
TAG=final_r3b bash tools/sessions/final_r3.sh tests && TAG=final_r3b bash tools/sessions/final_r3.sh bench
