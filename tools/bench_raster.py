"""Rasterizer phase timing (HIP events around each kernel of tsplat_raster_fwd) on the bench's
raster-only workload (1 scene, G = 131,072, 3 target views at 256x256), optionally with the
render-kernel diagnostics of TSPLAT_RASTER_DIAG (2: key load + sort only, 3: key load
only, 4: no blending -- fetch + cull + compaction only; images are wrong in those modes, only
the times mean something)."""
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
ap.add_argument("--waves", action="store_true", help="per-wave cost distribution (diag 5)")
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
        if n:  # (raster_scan: folded into the scatter kernel in round 5)
            row.append(f"{k}={ms / n * 1e3:.1f}us")
    print(f"diag={d}: " + " ".join(row), flush=True)
os.environ["TSPLAT_RASTER_DIAG"] = "0"
if args.waves:
    os.environ["TSPLAT_RASTER_DIAG"] = "5"
    color = step()[0]
    torch.cuda.synchronize()
    os.environ["TSPLAT_RASTER_DIAG"] = "0"
    # one value per 8x8 block (= wave): [views, 3, H/8, 8, W/8, 8] -> block corner
    c = color.reshape(-1, 3, color.shape[-2] // 8, 8, color.shape[-1] // 8, 8)[:, :, :, 0, :, 0]
    cyc, ent, chk = (c[:, i].flatten().double().cpu() for i in range(3))
    q = torch.tensor([0.0, 0.1, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64)
    print("wave cycles   quantiles", [f"{x:.0f}" for x in torch.quantile(cyc, q)])
    print("entries blended       ", [f"{x:.0f}" for x in torch.quantile(ent, q)])
    print("chunks walked         ", [f"{x:.0f}" for x in torch.quantile(chk, q)])
    print("corr(cycles, entries) %.3f  corr(cycles, chunks) %.3f" % (
        torch.corrcoef(torch.stack([cyc, ent]))[0, 1], torch.corrcoef(torch.stack([cyc, chk]))[0, 1]))
