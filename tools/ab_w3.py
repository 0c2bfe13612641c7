"""bf16x3 Winograd timing on a few census shapes with the library TSPLAT_LIB points at (ablation
builds from tools/build_ablation_w3.sh); one line per shape and form."""
import os
import sys

import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
SHAPES = [(2, 128, 128, 64, 64), (2, 256, 128, 32, 32), (2, 32, 32, 256, 256), (2, 163, 168, 256, 256)]
FORMS = sys.argv[1:] or ["1", "2"]


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


tag = os.path.basename(os.environ.get("TSPLAT_LIB") or "base") + " st" + os.environ.get("TSPLAT_WINO3_STAGE", "auto")
with torch.no_grad():
    for (n, ci, co, h, w) in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
        res = []
        for f in FORMS:
            os.environ["TSPLAT_WINO3_FORM"] = f
            res.append(f"form {f} {timeit(lambda: K.conv3x3_wino(x, wt, None, precision='bf16x3')):7.1f}")
        print(f"{tag:12s} {(n, ci, co, h, w)}: " + "  ".join(res), flush=True)
