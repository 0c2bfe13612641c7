# A/B of the working-tree library against tools/lib_old.so (HEAD build) on one box
export PYTHONPATH=$PWD
O=gpurun_out/ablib; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
cp transplat_amd/libtransplat_hip.so /tmp/lib_new.so
for r in 1 2; do
  cp /tmp/lib_new.so transplat_amd/libtransplat_hip.so
  timeout -k 10 300 $B > $O/new$r.log 2>&1 || exit 1
  cp tools/lib_old.so transplat_amd/libtransplat_hip.so
  timeout -k 10 300 $B > $O/old$r.log 2>&1; rc=$?
  cp /tmp/lib_new.so transplat_amd/libtransplat_hip.so; [ $rc -eq 0 ] || exit $rc
done
for f in new1 old1 new2 old2; do echo $f $(tail -1 $O/$f.log | cut -c80-140); done
