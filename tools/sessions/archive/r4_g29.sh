#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4_g29
export PYTHONPATH=$(pwd)
for lib in prev cur; do
  if [ $lib = prev ]; then export TSPLAT_LIB=tools/_bin/prev.so; else unset TSPLAT_LIB; fi
  timeout -k 10 300 python -u -m pytest -q -s --timeout 200 -m gpu tests/test_reference_golden.py -k "encoder_gpu_vs_reference" > gpurun_out/r4_g29/enc_$lib.log 2>&1
  echo "$lib: $(grep 'encoder vs reference' gpurun_out/r4_g29/enc_$lib.log | tr '\n' ' ')"
done
