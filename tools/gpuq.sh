#!/bin/bash
# Submit one gpurun call, waiting out "no free slot / box" answers (exit 3 or status=transient: nothing
# ran, nothing charged); any other outcome ends it. usage: gpuq.sh <out-file> <timeout-s> '<command>'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 60; continue; fi
  echo "rc=$rc" >> "$out"
  exit $rc
done
echo "gave up waiting for a slot" >> "$out"
