"""Rasterizer phase timing (HIP events around each kernel of tsplat_raster_fwd) on the bench's
raster-only workload (1 scene, G = 131,072, 3 target views at 256x256), optionally with the
render-kernel diagnostics of TSPLAT_RASTER_DIAG (1: no sort, 2: key load + sort only, 3: key
load only; images are wrong in those modes, only the times mean something)."""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from bench import build_raster_workload  # noqa: E402
from transplat_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--diag", default="0,2,3")
args = ap.parse_args()
dev = torch.device("cuda:0")
step, info, _ = build_raster_workload(1, dev, 0)
for _ in range(3):
    step()
torch.cuda.synchronize()
for d in args.diag.split(","):
    os.environ["TSPLAT_RASTER_DIAG"] = d
    row = []
    for k in ("raster_preprocess", "raster_scan", "raster_scatter", "raster_render", "raster"):
        step()
        torch.cuda.synchronize()
        _lib.prof_enable(k)
        for _ in range(args.iters):
            step()
        ms, n = _lib.prof_read()
        _lib.prof_enable(None)
        row.append(f"{k}={ms / n * 1e3:.1f}us")
    print(f"diag={d}: " + " ".join(row), flush=True)
os.environ["TSPLAT_RASTER_DIAG"] = "0"
