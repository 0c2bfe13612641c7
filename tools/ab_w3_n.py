"""bf16x3 Winograd time vs batch for the refine U-Net's 32-channel 256^2 convolution (per-workgroup
fixed cost vs throughput): forms 1 / 2, n = 1, 2, 4, 8, graph-timed."""
import os

import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * n) * 1e3


with torch.no_grad():
    for c, hw in [(32, 256), (128, 64)]:
        for n in (1, 2, 4, 8):
            x = torch.randn(n, c, hw, hw, device=dev)
            wt = torch.randn(c, c, 3, 3, device=dev) * 0.05
            res = []
            for f in ("1", "2", "5"):
                os.environ["TSPLAT_WINO3_FORM"] = f
                res.append(f"form {f} {timeit(lambda: K.conv3x3_wino(x, wt, None, precision='bf16x3')):7.1f}")
            mb = 2 * x.numel() * 4 / 1e6
            print(f"{c}->{c} at {hw}^2, n={n} ({mb:.0f} MB in+out): " + "  ".join(res), flush=True)
