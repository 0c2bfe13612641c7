"""Winograd F(2x2, 3x3) fp32 MFMA convolution (tsplat_conv3x3_wino_f32_fwd) vs MIOpen (algorithm
search on) and, where it applies, the direct kernel, on the encoder's 3x3 / stride-1 shapes with
their calls per step (b = 1 scene), graph-timed. Direct-equivalent TFLOP/s = 2 n h w co ci 9 / t."""
import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
# n, ci, co, h, w, calls per step (tools: the e2e encoder's conv2d census)
SHAPES = [
    (2, 163, 168, 256, 256, 1), (2, 168, 84, 256, 256, 1), (2, 128, 128, 64, 64, 11), (2, 256, 128, 64, 64, 5),
    (2, 32, 32, 256, 256, 7), (2, 128, 128, 72, 72, 4), (2, 64, 64, 128, 128, 4), (2, 128, 32, 256, 256, 1),
    (2, 64, 32, 256, 256, 2), (2, 128, 64, 144, 144, 1), (2, 128, 256, 64, 64, 1), (2, 32, 64, 256, 256, 1),
    (2, 64, 32, 252, 252, 1), (2, 96, 96, 64, 64, 3), (2, 128, 128, 36, 36, 4), (2, 128, 128, 32, 32, 5),
    (2, 32, 32, 128, 128, 5), (2, 38, 32, 256, 256, 1), (1, 128, 128, 64, 64, 2), (2, 256, 128, 32, 32, 2),
    (2, 64, 32, 128, 128, 2), (2, 96, 128, 72, 72, 1), (2, 96, 128, 64, 64, 1),
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
print(f"{'miopen':>8s} {'wino':>8s} {'GFLOP':>6s} {'TF/s':>6s} calls  shape (n, ci, co, h, w)")
with torch.no_grad():
    for (n, ci, co, h, w, calls) in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * (1.0 / (9 * ci) ** 0.5)
        b = torch.randn(co, device=dev)
        t1 = timeit(lambda: F.conv2d(x, wt, b, 1, 1))
        t2 = timeit(lambda: K.conv3x3_wino(x, wt, b))
        ref = F.conv2d(x, wt, b, 1, 1)
        err = ((K.conv3x3_wino(x, wt, b) - ref).abs().max() / ref.abs().max()).item()
        gf = 2.0 * n * h * w * co * ci * 9 / 1e9
        tot[0] += t1 * calls
        tot[1] += min(t1, t2) * calls
        print(f"{t1:8.1f} {t2:8.1f} {gf:6.2f} {gf / t2 * 1e3:6.1f} {calls:5d}  {(n, ci, co, h, w)} rel.err={err:.1e}",
              flush=True)
    # the to_gaussians head reads its input concatenation (refine_out, images, projected features) in
    # place: the same 163 -> 168 conv through the multi-source entry point
    parts = [torch.randn(2, c, 256, 256, device=dev) for c in (32, 3, 128)]
    wt = torch.randn(168, 163, 3, 3, device=dev) * (1.0 / (9 * 163) ** 0.5)
    b = torch.randn(168, device=dev)
    t2 = timeit(lambda: K.conv3x3_wino(parts[0], wt, b, extra=tuple(parts[1:])))
    ref = F.conv2d(torch.cat(parts, 1), wt, b, 1, 1)
    err = ((K.conv3x3_wino(parts[0], wt, b, extra=tuple(parts[1:])) - ref).abs().max() / ref.abs().max()).item()
    print(f"{'':8s} {t2:8.1f}  (2, 32+3+128, 168, 256, 256) read in place, rel.err={err:.1e}")
print(f"total per step: miopen {tot[0]:.1f} us, best-of {tot[1]:.1f} us")
