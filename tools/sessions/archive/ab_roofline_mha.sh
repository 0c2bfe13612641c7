export PYTHONPATH=$PWD
O=gpurun_out/rf; mkdir -p $O
for r in 1 2; do
  TSPLAT_MHA=16 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/m16_$r.log 2>&1 || exit 1
  TSPLAT_MHA=32 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/m32_$r.log 2>&1 || exit 1
done
for f in m16_1 m32_1 m16_2 m32_2; do tail -1 $O/$f.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$f',round(d['value'],1),round(r['frac'],4),round(r['avg_launch_ms']*1000,1))"; done
