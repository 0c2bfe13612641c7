O=gpurun_out/abrs2; mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  (export PYTHONPATH=$PWD; timeout -k 10 300 $B > $O/new$r.log 2>&1) || exit 1
  (cd tools/abold && export PYTHONPATH=$PWD && timeout -k 10 300 $B > ../../$O/old$r.log 2>&1) || exit 1
done
for f in new1 old1 new2 old2; do echo $f $(tail -1 $O/$f.log | grep -o '"value": [0-9.]*'); done
