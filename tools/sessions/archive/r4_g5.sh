#!/bin/bash
# Round 4: module goldens in both dense precisions (incl. the NCHW bf16x3 DPT head), then the C2
# A/B and profile of r4_g4.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_modules.py tests/test_conv.py tests/test_reference_golden.py tests/test_e2e.py -k "gpu or relu_in or bf16x3_step" -m gpu > gpurun_out/r4/pytest_g5.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r4/pytest_g5.log | head; tail -3 gpurun_out/r4/pytest_g5.log; exit 1; }
tail -1 gpurun_out/r4/pytest_g5.log
TAG=r4_g5 bash tools/sessions/r4_g4.sh
