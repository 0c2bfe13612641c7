"""Phase ablation of the few-channel conv kernel (TSPLAT_FEW_ABL: 1 no input loads, 2 no MFMAs, 4 no
stores, read per launch), HIP-event averages: python tools/few_abl.py n ci co h w"""
import os
import sys

import torch

from transplat_amd import kernels as K

n, ci, co, h, w = (int(v) for v in sys.argv[1:6])
dev = torch.device("cuda:0")
x = torch.randn(n, ci, h, w, device=dev)
wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
b = torch.randn(co, device=dev)


def timeit(fn, k=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


with K.dense_precision("bf16x3"):
    for abl in ("0", "1", "2", "4", "3", "5", "6", "7"):
        os.environ["TSPLAT_FEW_ABL"] = abl
        print(f"({n},{ci}->{co},{h}x{w}) abl {abl}: {timeit(lambda: K.conv3x3_wino(x, wt, b)):6.1f} us", flush=True)
