"""Direct conv kernel (tsplat_conv2d_f32_fwd) vs MIOpen (algorithm search on, cat / upsample glue
included as the module path runs it) on the U-Nets' convolution shapes, graph-timed; `route` is
what the dispatch rules pick for the shape (wino = conv3x3_wino_ok, direct = conv2d_direct_ok,
else MIOpen). --scale 4 multiplies the batch (2 views x b = 1 -> b = 4 x 2 = 8 maps; C2 b = 8)."""
import argparse

import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=1, help="batch multiplier for every shape")
args = ap.parse_args()
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
# n, c1, c2, h, w, cout, k, stride, upsample, calls per step
SHAPES = [
    (2, 128, 0, 16, 16, 128, 3, 1, False, 8), (2, 128, 128, 16, 16, 128, 3, 1, False, 2),
    (2, 128, 128, 16, 16, 128, 1, 1, False, 2), (2, 128, 0, 32, 32, 128, 3, 1, False, 4),
    (2, 128, 0, 64, 64, 128, 3, 2, False, 1), (2, 128, 0, 32, 32, 128, 3, 2, False, 1),
    (2, 128, 0, 16, 16, 128, 3, 1, True, 1), (2, 128, 128, 32, 32, 128, 3, 1, False, 2),
    (2, 128, 128, 32, 32, 128, 1, 1, False, 2), (2, 128, 0, 64, 64, 128, 3, 1, False, 3),
    (2, 128, 128, 64, 64, 128, 3, 1, False, 3), (2, 128, 0, 32, 32, 128, 3, 1, True, 1),
    (2, 32, 0, 16, 16, 32, 3, 1, False, 8), (2, 32, 32, 16, 16, 32, 3, 1, False, 2),
    (2, 32, 0, 32, 32, 32, 3, 1, False, 4), (2, 32, 32, 32, 32, 32, 3, 1, False, 2),
    (2, 32, 0, 64, 64, 32, 3, 1, False, 4), (2, 32, 32, 64, 64, 32, 3, 1, False, 2),
    (2, 32, 0, 128, 128, 32, 3, 1, False, 4), (2, 32, 32, 128, 128, 32, 3, 1, False, 2),
    (2, 32, 0, 256, 256, 32, 3, 2, False, 1), (2, 32, 0, 128, 128, 32, 3, 2, False, 1),
    (2, 32, 0, 64, 64, 32, 3, 2, False, 1), (2, 32, 0, 32, 32, 32, 3, 2, False, 1),
    (2, 32, 0, 16, 16, 32, 3, 1, True, 1), (2, 32, 0, 32, 32, 32, 3, 1, True, 1),
    (2, 32, 0, 64, 64, 32, 3, 1, True, 1), (2, 32, 32, 16, 16, 32, 1, 1, False, 2),
    (2, 32, 32, 32, 32, 32, 1, 1, False, 2), (2, 32, 32, 64, 64, 32, 1, 1, False, 2),
    (2, 32, 32, 128, 128, 32, 1, 1, False, 2), (2, 32, 32, 256, 256, 32, 3, 1, False, 2),
]


def timeit(fn, n=20):
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


tot = [0.0, 0.0]
print(f"{'miopen':>8s} {'direct':>8s} {'GFLOP':>6s} {'TF/s':>6s} calls  route  shape")
with torch.no_grad():
    for (n, c1, c2, h, w, co, k, st, up, calls) in SHAPES:
        n *= args.scale
        x1 = torch.randn(n, c1, h, w, device=dev)
        x2 = torch.randn(n, c2, h, w, device=dev) if c2 else None
        wt = torch.randn(co, c1 + c2, k, k, device=dev) * 0.05
        b = torch.randn(co, device=dev)

        def ref():
            x = x1 if x2 is None else torch.cat([x1, x2], 1)
            if up:
                x = F.interpolate(x, scale_factor=2, mode="nearest")
            return F.conv2d(x, wt, b, st, k // 2)

        t1 = timeit(ref)
        t2 = timeit(lambda: K.conv2d_direct(x1, wt, b, st, x2=x2, upsample=up))
        err = (K.conv2d_direct(x1, wt, b, st, x2=x2, upsample=up) - ref()).abs().max().item()
        hh, ww = (2 * h, 2 * w) if up else (h, w)
        gf = 2.0 * n * (hh // st) * (ww // st) * co * (c1 + c2) * k * k / 1e9
        route = ("wino" if not up and K.conv3x3_wino_ok(x1, wt, st, k // 2, extra=(x2,) if x2 is not None else ())
                 else "direct" if K.conv2d_direct_ok(x1, wt, st, c2=c2, upsample=up) else "miopen")
        tot[0] += t1 * calls
        tot[1] += t2 * calls
        print(f"{t1:8.1f} {t2:8.1f} {gf:6.3f} {gf / t2 * 1e3:6.1f} {calls:5d}  {route:6s} "
              f"{(n, c1, c2, h, w, co, k, st, up)} err={err:.1e}", flush=True)
print(f"total per step: miopen {tot[0]:.1f} us, direct {tot[1]:.1f} us")
