#!/bin/bash
# Diagnostic build of the library whose fp32 x32 window-attention kernel stamps per-workgroup phase
# clocks and hardware ids (TSPLAT_WA_STAMP=1, csrc/winattn.hip); output tools/_bin/wastamp.so, loaded
# via TSPLAT_LIB (tools/wa_stamps.py).
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p tools/_bin
OBJS=$(ls build/hip/*.o | grep -v winattn)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude -DTSPLAT_WA_STAMP=1 \
  -c transplat_amd/csrc/winattn.hip -o tools/_bin/winattn_stamp.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_bin/wastamp.so tools/_bin/winattn_stamp.o $OBJS
