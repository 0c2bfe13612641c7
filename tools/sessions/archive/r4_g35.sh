#!/bin/bash
# g35: the 7x7 / stride-2 stem on tsplat_conv2d_stem_f32_fwd: tests (kernel, backbone / encoder goldens),
# microbenchmark vs MIOpen (default and deterministic solvers), C2 vs the previous library and C2 with
# --conv-deterministic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4_g35
mkdir -p $OUT
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_conv.py \
  tests/test_modules.py tests/test_reference_golden.py -k "stem or backbone or encoder_gpu" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
grep -E "stem \(|encoder vs|passed|failed" $OUT/pytest.log | tail -12
timeout -k 10 120 python -u - > $OUT/stem_bench.log 2>&1 <<'PY' || { tail -5 $OUT/stem_bench.log; exit 3; }
import torch, torch.nn.functional as F
from transplat_amd import kernels as K
dev = torch.device("cuda:0")
x = torch.randn(2, 3, 256, 256, device=dev); w = torch.randn(64, 3, 7, 7, device=dev) * 0.08
def t(fn, n=50):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n * 1e3
for det in (False, True):
    torch.backends.cudnn.benchmark = True; torch.backends.cudnn.deterministic = det
    print(f"MIOpen (deterministic={det}): {t(lambda: F.conv2d(x, w, None, 2, 3)):.1f} us")
print(f"tsplat stem: {t(lambda: K.conv2d_stem(x, w)):.1f} us")
PY
cat $OUT/stem_bench.log | grep -v amdgpu
for i in 1 2; do
  for v in prev cur curdet; do
    extra=""; unset TSPLAT_LIB
    [ $v = prev ] && export TSPLAT_LIB=tools/_bin/prev.so
    [ $v = curdet ] && extra="--conv-deterministic"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $extra > $OUT/bench_c2_${v}_$i.log 2>&1 || { tail -5 $OUT/bench_c2_${v}_$i.log; exit 4; }
    echo "$v $i c2 $(tail -1 $OUT/bench_c2_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), d["ms_per_step"])')"
  done
done
