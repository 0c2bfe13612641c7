"""Graph-timed bf16x3 Winograd launch per workgroup form for given shapes:
python tools/wino3_forms.py "n,ci,co,h,w" ... (forms 1-6 via TSPLAT_WINO3_FORM, FORMS=0,1,..., read per launch)."""
import os
import sys

import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
for spec in sys.argv[1:]:
    n, ci, co, h, w = (int(a) for a in spec.split(","))
    x = torch.randn(n, ci, h, w, device=dev)
    wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
    row = []
    for form in os.environ.get("FORMS", "0,1,2,3,4,5,6").split(","):
        os.environ["TSPLAT_WINO3_FORM"] = form
        s = torch.cuda.Stream()
        try:
            with torch.cuda.stream(s), torch.no_grad():
                for _ in range(3):
                    K.conv3x3_wino(x, wt, None, precision="bf16x3")
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s), torch.no_grad():
                for _ in range(10):
                    K.conv3x3_wino(x, wt, None, precision="bf16x3")
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            row.append(f"form{form} {e0.elapsed_time(e1) * 1e3 / 50:7.1f}")
        except RuntimeError as e:
            row.append(f"form{form} n/a")
    os.environ.pop("TSPLAT_WINO3_FORM", None)
    print(spec, " | ".join(row), flush=True)
