#!/bin/bash
# Diagnostic builds of the library with one phase of the key-pair attention loop removed
# (TSPLAT_WA_ABL=N, see csrc/winattn.hip); output build/abl/libN.so, loaded via TSPLAT_LIB.
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p build/abl
OBJS=$(ls build/hip/*.o | grep -v winattn)
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -DTSPLAT_WA_ABL=$n -c transplat_amd/csrc/winattn.hip -o build/abl/winattn$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/lib$n.so build/abl/winattn$n.o $OBJS
done
