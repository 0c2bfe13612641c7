"""Census of the direct-kernel convolutions (kernels.conv2d_direct) of one e2e step: the shapes one
eager step launches (with their inputs), then each shape graph-timed alone (20 calls per replay, as
the step's hipGraph launches them). python tools/direct_census.py [dense_dtype]"""
import sys
from collections import Counter

import torch

from transplat_amd import kernels as K
from transplat_amd import streams
from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

dense = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
dev = torch.device("cuda:0")
model = build_model(dev, dense)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
orig = K.conv2d_direct
calls = Counter()
args = {}


def logged(x1, weight, bias=None, stride=1, x2=None, upsample=False):
    n, c1, h, w = x1.shape
    c2 = x2.shape[1] if x2 is not None else 0
    key = (n, c1, c2, h, w, weight.shape[0], weight.shape[-1] if weight.dim() == 4 else 1, stride, bool(upsample))
    calls[key] += 1
    if key not in args:
        args[key] = tuple(t.clone() if torch.is_tensor(t) else t for t in (x1, weight, bias, stride, x2, upsample))
    return orig(x1, weight, bias, stride, x2, upsample)


K.conv2d_direct = logged
with torch.no_grad(), streams.serial():
    model.test_step(data)
    calls.clear()
    model.test_step(data)
K.conv2d_direct = orig
rows = []
s = torch.cuda.Stream()
prec = K.dense_precision(dense) if dense in ("bf16x3",) else torch.no_grad()
prec.__enter__()  # the step's dense mode (bf16x3: the split-bf16 direct kernel unless TSPLAT_CONV_X3=0)
for key, a in args.items():
    with torch.cuda.stream(s):
        for _ in range(3):
            orig(*a)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(20):
            orig(*a)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    rows.append((key, e0.elapsed_time(e1) * 1e3 / 100))
tot = 0.0
for key, t in sorted(rows, key=lambda r: -r[1] * calls[r[0]]):
    c = calls[key]
    tot += t * c
    n, c1, c2, h, w, co, k, st, up = key
    fl = 2.0 * n * (h * (2 if up else 1) // st) * (w * (2 if up else 1) // st) * co * (c1 + c2) * k * k
    print(f"{c:3d} x {t:6.1f} us = {t * c:6.1f}  n{n} ci {c1}+{c2} {h}x{w} -> co {co} k{k} s{st}{' up' if up else ''}"
          f"  {fl / 1e9:6.3f} GFLOP  {fl / (t * 1e-6) / 1e12:6.1f} TF/s")
print(f"total {tot:.1f} us over {sum(calls.values())} calls ({dense})")
