export PYTHONPATH=$PWD
O=gpurun_out/dom; mkdir -p $O
for k in uv_coarse uv_cross_table; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dominant $k > $O/$k.log 2>&1 || exit 1
tail -1 $O/$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$k', d['value'], r['avg_launch_ms'], r['achieved'], r['frac'])"
done
cp transplat_amd/libtransplat_hip.so /tmp/lib_new.so && cp tools/lib_old.so transplat_amd/libtransplat_hip.so
k=uv_coarse; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dominant $k > $O/${k}_old.log 2>&1; rc=$?
cp /tmp/lib_new.so transplat_amd/libtransplat_hip.so; [ $rc -eq 0 ] || exit $rc
tail -1 $O/${k}_old.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('old $k', d['value'], r['avg_launch_ms'], r['achieved'], r['frac'])"
