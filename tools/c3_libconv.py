"""The library convolutions left in a step (routes.record census), each unique shape timed on MIOpen
and on the hand-written routes that could take it (direct bf16x3 / exact fp32, Winograd bf16x3),
HIP-event averages of 20 calls after warmup. usage: c3_libconv.py [batch] [dense] [attn]"""
import collections
import sys

import torch
import torch.nn.functional as F

from transplat_amd import kernels as K
from transplat_amd import routes
from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dense = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
attn = sys.argv[3] if len(sys.argv) > 3 else "bf16"
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
model = build_model(dev, dense, attn_dtype=attn)
data = S.make_batch(batch, image_shape=(256, 256), device=dev)
with torch.no_grad():
    model.test_step(data)
    with routes.record() as r:  # run with TSPLAT_CONV_LIBFREE_X3=0 to list what reaches MIOpen without it
        model.test_step(data)
torch.cuda.synchronize()
convs = collections.Counter()
for op, arith, shapes in r.library:
    if op in routes._GEMMS:
        continue
    x, w = shapes[0], shapes[1]
    st, pad, tr = shapes[-1]
    convs[(x, w, len(shapes) == 4, st, pad, tr, arith)] += 1


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


tot = 0.0
for (x, w, has_b, st, pad, tr, arith), n in sorted(convs.items(), key=lambda kv: -kv[1]):
    xi = torch.randn(x, device=dev)
    wi = torch.randn(w, device=dev) * 0.05
    bi = torch.randn(w[0], device=dev) if has_b else None
    row = f"{n:2d} x  x={x} w={w} stride={st} pad={pad} {arith}:"
    if tr:
        print(row, "transposed (skipped)")
        continue
    t_mi = timeit(lambda: F.conv2d(xi, wi, bi, st, pad))
    tot += n * t_mi
    row += f" MIOpen {t_mi:7.1f} us"
    k = w[2]
    if w[2] == w[3] and st[0] == st[1] and pad[0] == k // 2 and k in (1, 3):
        with K.dense_precision("bf16x3"):
            y0 = F.conv2d(xi, wi, bi, st, pad)
            y1 = K.conv2d_direct(xi, wi, bi, st[0])
            err = ((y1 - y0).abs().max() / y0.abs().max()).item()
            row += f" | direct-x3 {timeit(lambda: K.conv2d_direct(xi, wi, bi, st[0])):7.1f} us (err {err:.1e})"
            if k == 3 and st[0] == 1:
                row += f" | wino-x3 {timeit(lambda: K.conv3x3_wino(xi, wi, bi)):7.1f} us"
        row += f" | direct-f32 {timeit(lambda: K.conv2d_direct(xi, wi, bi, st[0])):7.1f} us"
    print(row, flush=True)
print(f"MIOpen total {tot:.1f} us per step ({sum(convs.values())} calls)")
