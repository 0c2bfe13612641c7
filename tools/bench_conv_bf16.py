"""Per-shape timing of the bf16 implicit-GEMM convolution (kernels.conv_bf16) against F.conv2d under
bf16 autocast (MIOpen) for the C3 step's convolution shapes (profiles/r3/probe/ops_c3.log).
Usage: python tools/bench_conv_bf16.py [--iters 20]"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from transplat_amd import kernels as K  # noqa: E402

SHAPES = [  # n, ci, h, w, co, k, up, src dtype
    (16, 32, 256, 256, 32, 3, False, "bf16"),
    (16, 128, 64, 64, 128, 3, False, "bf16"),
    (16, 256, 64, 64, 128, 3, False, "bf16"),
    (16, 64, 128, 128, 64, 3, False, "bf16"),
    (16, 96, 64, 64, 96, 3, False, "bf16"),
    (16, 128, 16, 16, 128, 3, False, "bf16"),
    (16, 32, 16, 16, 32, 3, False, "bf16"),
    (16, 128, 32, 32, 128, 3, False, "bf16"),
    (16, 256, 64, 64, 128, 1, False, "bf16"),
    (16, 128, 32, 32, 128, 3, True, "bf16"),
    (16, 64, 256, 256, 32, 3, False, "f32"),
    (16, (32, 3, 128), 256, 256, 168, 3, False, "mix"),  # to_gaussians conv 1 on the concat (GELU after)
    (16, 168, 256, 256, 84, 3, False, "bf16"),           # to_gaussians conv 2
    (16, 32, 256, 256, 64, 3, False, "bf16"),            # to_disparity conv 1
]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
print(f"{'shape':44s} {'hip us':>8s} {'miopen us':>10s} {'TF/s':>7s}", flush=True)
for n, ci, h, w, co, k, up, sdt in SHAPES:
    hs, ws = (h // 2, w // 2) if up else (h, w)
    chans = ci if isinstance(ci, tuple) else (ci,)
    dts = [torch.float32 if (sdt == "f32" or (sdt == "mix" and i > 0)) else torch.bfloat16 for i in range(len(chans))]
    xs = [torch.randn(n, c, hs, ws, device=dev).to(d) for c, d in zip(chans, dts)]
    ci = sum(chans)
    wt = torch.randn(co, ci, k, k, device=dev) * 0.05
    b = torch.randn(co, device=dev)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        hip = timed(lambda: K.conv_bf16(xs[0], wt, b, extra=tuple(xs[1:]), upsample=up), args.iters)

        def ref():
            x = torch.cat(xs, 1) if len(xs) > 1 else xs[0]
            return F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest") if up else x, wt, b, padding=k // 2)
        mio = timed(ref, args.iters)
    flop = 2.0 * n * h * w * co * ci * k * k
    tag = f"{n}x{ci}x{h}x{w}->{co} k{k}{' up' if up else ''} {sdt}"
    print(f"{tag:44s} {hip:8.1f} {mio:10.1f} {flop / hip / 1e6:7.1f}", flush=True)
