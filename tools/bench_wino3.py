"""bf16x3 Winograd (tsplat_conv3x3_wino_bf16x3_fwd) vs the exact-fp32 Winograd kernel on the C2 step's
3x3 census (tools/bench_wino.py SHAPES), graph-timed: per shape the fp32 kernel, the bf16x3 launch's
own form and each forced form (TSPLAT_WINO3_FORM 1-4), the call-weighted step totals, and the max
relative error of both precisions against float64 conv2d.
usage: bench_wino3.py [--quick]"""
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

src = Path(__file__).with_name("bench_wino.py").read_text()
SHAPES = eval(src.split("SHAPES = ", 1)[1].split("\n]\n", 1)[0] + "\n]")
dev = torch.device("cuda:0")
FORMS = ["auto"] if "--quick" in sys.argv else ["auto", "1", "2", "4", "5"]


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


tot = {k: 0.0 for k in ["fp32"] + FORMS}
print("times in us; calls; shape (n, ci, co, h, w); rel. err fp32 / bf16x3(auto)")
print(f"{'fp32':>8s} " + " ".join(f"{'x3:' + f:>8s}" for f in FORMS))
with torch.no_grad():
    for (n, ci, co, h, w, calls) in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * (1.0 / (9 * ci) ** 0.5)
        b = torch.randn(co, device=dev)
        ref = F.conv2d(x.double(), wt.double(), b.double(), 1, 1)
        t = {"fp32": timeit(lambda: K.conv3x3_wino(x, wt, b, precision="fp32"))}
        for f in FORMS:
            if f == "auto":
                os.environ.pop("TSPLAT_WINO3_FORM", None)
            else:
                os.environ["TSPLAT_WINO3_FORM"] = f
            t[f] = timeit(lambda: K.conv3x3_wino(x, wt, b, precision="bf16x3"))
        os.environ.pop("TSPLAT_WINO3_FORM", None)
        e32 = ((K.conv3x3_wino(x, wt, b, precision="fp32").double() - ref).abs().max() / ref.abs().max()).item()
        e3 = ((K.conv3x3_wino(x, wt, b, precision="bf16x3").double() - ref).abs().max() / ref.abs().max()).item()
        for k in tot:
            tot[k] += t[k] * calls
        print(f"{t['fp32']:8.1f} " + " ".join(f"{t[f]:11.1f}" for f in FORMS)
              + f"  {calls:3d}  {(n, ci, co, h, w)}  {e32:.1e} / {e3:.1e}", flush=True)
print("step totals (us): " + ", ".join(f"{k} {v:.1f}" for k, v in tot.items()))
