#!/bin/bash
# Round-3 A/B: cost-balanced raster render order (TSPLAT_RASTER_BAL) and the one-workgroup-per-CU
# fp32 window-attention form (TSPLAT_WA_OCC1): GPU tests of both, per-kernel A/Bs, C2 same-box A/B
# (both off vs both on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/${TAG:-r3e}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_raster.py tests/test_reference_golden.py tests/test_encoder_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for b in 0 1; do
  TSPLAT_RASTER_BAL=$b timeout -k 10 120 python tools/bench_raster.py --diag 0 --iters 50 > $OUT/phases_bal${b}_$r.log 2>&1 || exit 1
  echo "bal=$b $(grep diag= $OUT/phases_bal${b}_$r.log)"
done; done
TSPLAT_RASTER_BAL=0 timeout -k 10 120 python tools/bench_raster.py --diag 0 --iters 5 --waves > $OUT/waves_bal0.log 2>&1 || exit 1
TSPLAT_RASTER_BAL=1 timeout -k 10 120 python tools/bench_raster.py --diag 0 --iters 5 --waves > $OUT/waves_bal1.log 2>&1 || exit 1
grep -h "quantiles" $OUT/waves_bal0.log $OUT/waves_bal1.log
for r in 1 2; do for o in 0 1; do for sh in 0 1; do
  TSPLAT_WA_OCC1=$o timeout -k 10 60 python tools/bench_winattn.py --batch 2 --shift $sh --iters 100 > $OUT/wa_occ${o}_sh${sh}_$r.log 2>&1 || exit 1
  echo "occ1=$o shift=$sh $(tail -1 $OUT/wa_occ${o}_sh${sh}_$r.log)"
done; done; done
for r in 1 2; do for b in 0 1; do
  TSPLAT_RASTER_BAL=$b TSPLAT_WA_OCC1=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_new${b}_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" $OUT/c2_new${b}_$r.log
done; done
echo done
