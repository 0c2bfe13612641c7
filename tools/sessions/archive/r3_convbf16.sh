#!/bin/bash
# bf16 implicit-GEMM conv: tests, per-shape timing vs MIOpen (+ rocprof kernel times), C3 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-convbf16}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -q --timeout 280 -k "bf16" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -25 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/bench_conv_bf16.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
grep -v amdgpu.ids $OUT/bench.log
TSPLAT_CONVBF16_BIG=0 timeout -k 10 300 python tools/bench_conv_bf16.py > $OUT/bench_nobig.log 2>&1 || { echo "bench nobig failed"; exit 1; }
echo "big off"; grep -v amdgpu.ids $OUT/bench_nobig.log | tail -n +2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/tools/bench_conv_bf16.py --iters 5 > $OUT/prof.log 2>&1 || { echo prof failed; exit 1; }
cd $R
run() {
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py $extra --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]:24s} {d['value']:8.1f} views/s {d['ms_per_step']:7.3f} ms  attn {d['roofline']['frac']:.3f}")
PY
}
C3="--batch 8 --dense-dtype bf16"
run c3 "$C3"
run c3_nobig "$C3" TSPLAT_CONVBF16_BIG=0
run c3_noconv "$C3" TSPLAT_CONV_BF16=0
run c3b "$C3"
echo done
