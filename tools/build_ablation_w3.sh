#!/bin/bash
# Diagnostic builds of the library with one phase of the bf16x3 Winograd loop removed
# (TSPLAT_W3_ABL=N, see csrc/winoconv3.hip: 1 no patch loads, 2 no MFMAs, 3 no A loads);
# output tools/_bin/w3ablN.so, loaded via TSPLAT_LIB (tools/ab_w3.py).
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p tools/_bin
OBJS=$(ls build/hip/*.o | grep -v winoconv3)
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude -DTSPLAT_W3_ABL=$n \
    -c transplat_amd/csrc/winoconv3.hip -o tools/_bin/winoconv3_abl$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_bin/w3abl$n.so tools/_bin/winoconv3_abl$n.o $OBJS
done
