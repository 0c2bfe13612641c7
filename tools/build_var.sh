#!/bin/bash
# Variant build of the HIP library for same-box A/Bs (TSPLAT_LIB=<out>): one source recompiled with
# extra flags (or taken from a git revision: SRC_REV=<rev>), the other objects from build/hip/.
# usage: build_var.sh <out.so> <file.hip> [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
OUT=$1; F=$2; shift 2
mkdir -p "$(dirname "$OUT")" build/var
STEM=$(basename "$F" .hip)
SRC=transplat_amd/csrc/$F
if [ -n "$SRC_REV" ]; then git show "$SRC_REV:transplat_amd/csrc/$F" > build/var/$F; SRC=build/var/$F; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude -Itransplat_amd/csrc "$@" -c $SRC -o build/var/$STEM.o
OBJS=$(ls build/hip/*.o | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS build/var/$STEM.o
echo "$OUT"
