#!/bin/bash
# Diagnostic build with per-wave s_memtime segment stamps in the window-attention kernels
# (TSPLAT_WA_STAMP=1): build/abl/lib_stamp.so, loaded via TSPLAT_LIB. Never the shipped library.
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p build/abl
OBJS=$(ls build/hip/*.o | grep -v winattn)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -DTSPLAT_WA_STAMP=1 -c transplat_amd/csrc/winattn.hip -o build/abl/winattn_stamp.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/lib_stamp.so build/abl/winattn_stamp.o $OBJS
