#!/bin/bash
# Two-key-halves fp32 window attention (TSPLAT_WA_HALVES): attention / module GPU tests, kernel A/B
# (b = 2 views, unshifted / shifted), C2 same-box A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$(pwd)
OUT=gpurun_out/${TAG:-r3f}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_encoder_ops.py tests/test_modules.py tests/test_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for o in 0 1; do for sh in 0 1; do
  TSPLAT_WA_HALVES=$o timeout -k 10 60 python tools/bench_winattn.py --batch 2 --shift $sh --iters 100 > $OUT/wa_halves${o}_sh${sh}_$r.log 2>&1 || exit 1
  echo "halves=$o shift=$sh $(tail -1 $OUT/wa_halves${o}_sh${sh}_$r.log)"
done; done; done
for r in 1 2; do for o in 0 1; do
  TSPLAT_WA_HALVES=$o timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_halves${o}_$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms']*1e3,1))" $OUT/c2_halves${o}_$r.log
done; done
echo done
