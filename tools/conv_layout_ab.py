"""Time every distinct convolution of one e2e step in NCHW and in channels-last (NHWC) layout,
MIOpen algorithm search on, to see where a channels-last chain would pay.
usage: conv_layout_ab.py [--dense-dtype fp32]"""
import argparse
import traceback
from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

ap = argparse.ArgumentParser()
ap.add_argument("--dense-dtype", default="fp32")
args = ap.parse_args()
dev = torch.device("cuda:0")
model = build_model(dev, args.dense_dtype)
shapes = OrderedDict()


class _Rec(TorchFunctionMode):
    """Records every conv2d call (module or functional) with its site."""

    def __torch_function__(self, func, types, a=(), kw=None):
        kw = kw or {}
        if func is F.conv2d:
            x, w = a[0], a[1]
            b = a[2] if len(a) > 2 else kw.get("bias")
            st = a[3] if len(a) > 3 else kw.get("stride", 1)
            pd = a[4] if len(a) > 4 else kw.get("padding", 0)
            g = a[6] if len(a) > 6 else kw.get("groups", 1)
            site = next((f"{f.filename.split('/')[-1]}:{f.lineno}" for f in reversed(traceback.extract_stack()[:-1])
                         if "transplat_amd" in f.filename and "torch" not in f.filename), "?")
            key = (tuple(x.shape), tuple(w.shape), tuple(st) if isinstance(st, (list, tuple)) else st,
                   tuple(pd) if isinstance(pd, (list, tuple)) else pd, g, b is not None, x.is_contiguous(), x.dtype)
            shapes.setdefault(key, []).append(site)
        return func(*a, **kw)


data = S.make_batch(1, image_shape=(256, 256), device=dev)
with torch.no_grad(), _Rec():
    model.test_step(data)
torch.cuda.synchronize()
torch.backends.cudnn.benchmark = True


def timeit(fn, n=20):
    """GPU time per call from a captured graph of n calls (no host launch overhead)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * n) * 1e3


tot = [0.0, 0.0, 0.0]
print(f"{'NCHW us':>8s} {'NHWC us':>8s} {'+conv us':>8s} {'calls':>5s}  input weight stride pad  sites")
with torch.no_grad():
    for (xs, ws, st, pd, g, hb, contig, dt), sites in shapes.items():
        x = torch.randn(xs, device=dev, dtype=dt)
        w = torch.randn(ws, device=dev, dtype=dt) * 0.01
        b = torch.randn(ws[0], device=dev, dtype=dt) if hb else None
        t1 = timeit(lambda: F.conv2d(x, w, b, st, pd, 1, g))
        xc, wc = x.contiguous(memory_format=torch.channels_last), w.contiguous(memory_format=torch.channels_last)
        t2 = timeit(lambda: F.conv2d(xc, wc, b, st, pd, 1, g))
        # NHWC conv entered and left from NCHW tensors (layout copies included)
        t3 = timeit(lambda: F.conv2d(x.contiguous(memory_format=torch.channels_last), wc, b, st, pd, 1, g).contiguous())
        n = len(sites)
        for i, t in enumerate((t1, t2, t3)):
            tot[i] += t * n
        print(f"{t1:8.1f} {t2:8.1f} {t3:8.1f} {n:5d}  {xs} {ws} s{st} p{pd} contig={contig}  {sorted(set(sites))}",
              flush=True)
print(f"total per step: NCHW {tot[0]:.1f} us, NHWC {tot[1]:.1f} us, NHWC+copies {tot[2]:.1f} us")
