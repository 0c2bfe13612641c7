"""Census of the 3x3 Winograd launches of one eager e2e step (shape, precision, the bf16x3 launch
form), with per-call HIP-event times: python tools/wino_census.py [dense_dtype] [batch]."""
import sys
from collections import Counter

import torch

from transplat_amd import kernels as K
from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

dense = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda:0")
model = build_model(dev, dense)
data = S.make_batch(batch, image_shape=(256, 256), device=dev)
orig = K.conv3x3_wino
calls = Counter()
times = Counter()


def logged(x, weight, *a, **kw):
    n, _, h, w = x.shape
    ci = x.shape[1] + sum(t.shape[1] for t in kw.get("extra", ()))
    key = (n, ci, weight.shape[0], h, w, x.is_contiguous(), bool(kw.get("relu_in")), kw.get("residual") is not None)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y = orig(x, weight, *a, **kw)
    e1.record()
    e1.synchronize()
    calls[key] += 1
    times[key] += e0.elapsed_time(e1) * 1e3
    return y


K.conv3x3_wino = logged
with torch.no_grad():
    model.test_step(data)
    calls.clear()
    times.clear()
    model.test_step(data)
tot = 0.0
for key, c in sorted(calls.items(), key=lambda kv: -times[kv[0]]):
    tot += times[key]
    n, ci, co, h, w = key[:5]
    gf = 2.0 * n * ci * co * h * w * 9 / 1e9  # direct-equivalent FLOPs
    print(f"{c:3d} x {times[key] / c:7.1f} us {gf / (times[key] / c) * 1e3:6.1f} TF/s  "
          f"(n, ci, co, h, w, contiguous, relu_in, residual) = {key}")
print(f"total {tot:.1f} us over {sum(calls.values())} calls ({dense}, b = {batch})")
