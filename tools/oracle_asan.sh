#!/bin/bash
# The CPU rasterizer oracle tests under AddressSanitizer + UndefinedBehaviorSanitizer:
# oracle/raster_ref.c built with -fsanitize=address,undefined (make -C oracle asan), loaded by the
# ctypes front end through TSPLAT_ORACLE_LIB, the ASan runtime preloaded into python. Host code only.
set -e
cd "$(dirname "$0")/.."
make -s -C oracle asan
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export TSPLAT_ORACLE_LIB=$PWD/oracle/build/libtsplat_oracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export OMP_NUM_THREADS=1
LD_PRELOAD="$ASAN_RT $UBSAN_RT" python -m pytest -q -p no:cacheprovider tests/test_raster.py tests/test_reference_golden.py -m "not gpu" "$@"
