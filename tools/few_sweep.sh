export PYTHONPATH=$PWD
for tr in 8 4 2; do for ar in 0 1; do
  if [ $tr = 8 ] && [ $ar = 1 ]; then continue; fi
  echo "== TR=$tr AREG=$ar"
  TSPLAT_FEW_TR=$tr TSPLAT_FEW_AREG=$ar timeout -k 10 100 python tools/fewch_conv.py 2>&1 | grep -v amdgpu | grep few | cut -c1-120 || exit 1
done; done
