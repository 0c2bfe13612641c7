#!/bin/bash
# Build the HIP library of an earlier commit (default HEAD~1) into tools/_bin/prev.so, for same-box
# A/Bs through TSPLAT_LIB (the C-ABI must be unchanged between the two).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD~1}
TMP=$(mktemp -d)
git archive "$REV" transplat_amd/csrc include | tar -x -C "$TMP"
mkdir -p tools/_bin "$TMP/obj"
for f in "$TMP"/transplat_amd/csrc/*.hip; do
  extra=""
  case $(basename "$f") in raster.hip) extra="-fno-slp-vectorize" ;; upsample.hip) extra="-ffp-contract=off" ;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -I"$TMP/include" $extra -c "$f" -o "$TMP/obj/$(basename "$f" .hip).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_bin/prev.so "$TMP"/obj/*.o
rm -rf "$TMP"
echo "tools/_bin/prev.so <- $REV"
