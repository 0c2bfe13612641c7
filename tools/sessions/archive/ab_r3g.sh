#!/bin/bash
# Occupancy-4 register budget for the 4-wave Winograd kernel (TSPLAT_WINO_OCC4): per-shape A/B over
# the census (with the float64 error check), C2 same-box A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/${TAG:-r3g}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_wino.py TSPLAT_WINO_OCC4 0 1 > $OUT/ab_wino_occ4.log 2>&1; rc=$?
grep -v amdgpu $OUT/ab_wino_occ4.log | tail -26; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for o in 0 1; do
  TSPLAT_WINO_OCC4=$o timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_occ4${o}_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline_step_dominant']['frac'],4))" $OUT/c2_occ4${o}_$r.log
done; done
echo done
