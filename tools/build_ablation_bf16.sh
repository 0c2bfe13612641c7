#!/bin/bash
# Diagnostic builds of the library with one phase of the bf16 v2 attention loop removed
# (TSPLAT_WA2_ABL=N, see csrc/winattn.hip); output transplat_amd/abl/libN.so (travels to the GPU
# box), loaded via TSPLAT_LIB. Never the shipped library.
set -e
cd "$(dirname "$0")/.."
python -m transplat_amd.build > /dev/null
mkdir -p transplat_amd/abl
OBJS=$(ls build/hip/*.o | grep -v winattn)
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude -DTSPLAT_WA2_ABL=$n -c transplat_amd/csrc/winattn.hip -o build/abl2_winattn$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o transplat_amd/abl/lib$n.so build/abl2_winattn$n.o $OBJS
done
