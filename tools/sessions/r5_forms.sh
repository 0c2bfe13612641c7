#!/bin/bash
# Round-5 Winograd form probe: forced-form kernel tests for the new forms, then graph-timed forms
# per census shape (tools/wino3_forms.py; FORMS selects the columns).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r5_forms}
mkdir -p $OUT
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -q -k "${TESTK:-wino_bf16x3_kernel and 6}" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
FORMS=${FORMS:-0,1,2,4,6} timeout -k 10 400 python -u tools/wino3_forms.py ${SHAPES:-2,163,168,256,256 2,168,84,256,256 2,128,128,64,64 2,32,32,256,256 2,256,128,64,64 2,64,64,128,128 2,128,128,72,72 16,163,168,256,256 16,168,84,256,256 16,128,128,64,64 16,32,32,256,256} > $OUT/forms.log 2>&1 || { tail -5 $OUT/forms.log; exit 1; }
cat $OUT/forms.log
