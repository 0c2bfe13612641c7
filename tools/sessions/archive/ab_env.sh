# Same-box A/B of one environment knob on the C2 bench: bash tools/sessions/ab_env.sh VAR NEW OLD [bench args]
export PYTHONPATH=$PWD
VAR=$1; NEW=$2; OLD=$3; shift 3
O=gpurun_out/abenv; mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline $*"
for r in 1 2; do
  env $VAR=$NEW timeout -k 10 300 $B > $O/new$r.log 2>&1 || exit 1
  env $VAR=$OLD timeout -k 10 300 $B > $O/old$r.log 2>&1 || exit 1
done
for f in new1 old1 new2 old2; do echo $f $(tail -1 $O/$f.log | grep -o '"value": [0-9.]*'); done
