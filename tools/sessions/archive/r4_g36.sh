#!/bin/bash
# g36: tiny-map / long-reduction convolutions (the DPT's 768 -> 768 stride-2 3x3 at 18^2) on the direct kernel
# regardless of the FLOP cap (TSPLAT_CONV_SMALLMAP=1, default) vs MIOpen (=0): microbenchmark, DPT / encoder
# tests, C2 with MIOpen's default and deterministic solvers, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g36
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_modules.py \
  tests/test_reference_golden.py -k "depth_anything or encoder_gpu" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
grep -E "encoder vs|passed|failed" $OUT/pytest.log | tail -4
timeout -k 10 120 python -u - > $OUT/conv_bench.log 2>&1 <<'PY' || { tail -5 $OUT/conv_bench.log; exit 3; }
import torch, torch.nn.functional as F
from transplat_amd import kernels as K
dev = torch.device("cuda:0")
x = torch.randn(2, 768, 18, 18, device=dev); w = torch.randn(768, 768, 3, 3, device=dev) * 0.01; b = torch.randn(768, device=dev)
def t(fn, n=50):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n * 1e3
for det in (False, True):
    torch.backends.cudnn.benchmark = True; torch.backends.cudnn.deterministic = det
    print(f"MIOpen (deterministic={det}): {t(lambda: F.conv2d(x, w, b, 2, 1)):.1f} us")
ref = F.conv2d(x.double(), w.double(), b.double(), 2, 1)
y = K.conv2d_direct(x, w, b, 2)
print(f"direct kernel: {t(lambda: K.conv2d_direct(x, w, b, 2)):.1f} us, rel err {((y.double() - ref).abs().max() / ref.abs().max()).item():.2e}")
PY
grep -v amdgpu $OUT/conv_bench.log
for i in 1 2; do
  for sm in 0 1; do
    for det in 0 1; do
      extra=""; [ $det = 1 ] && extra="--conv-deterministic"
      TSPLAT_CONV_SMALLMAP=$sm timeout -k 10 300 python -u bench.py --no-cpu-baseline $extra > $OUT/bench_c2_${sm}${det}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${sm}${det}_$i.log; exit 4; }
      echo "smallmap $sm det $det $i c2 $(tail -1 $OUT/bench_c2_${sm}${det}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')"
    done
  done
done
