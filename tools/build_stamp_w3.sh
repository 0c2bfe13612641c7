#!/bin/bash
# Diagnostic build of the library whose bf16x3 Winograd kernels stamp per-workgroup phase clocks
# (TSPLAT_W3_STAMP=1, csrc/winoconv3.hip); output tools/_bin/w3stamp.so, loaded via TSPLAT_LIB
# (tools/w3_stamps.py).
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p tools/_bin
OBJS=$(ls build/hip/*.o | grep -v winoconv3)
for n in 1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude -DTSPLAT_W3_STAMP=1 \
    -c transplat_amd/csrc/winoconv3.hip -o tools/_bin/winoconv3_stamp.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_bin/w3stamp.so tools/_bin/winoconv3_stamp.o $OBJS
done
