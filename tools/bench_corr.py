"""Microbenchmark of the coarse correlation kernel alone at the production shape (64x64 feature
maps, 2 views, D = C = 128, the bench's synthetic cameras). Prints average us per call (HIP
events around the launches) and the HBM roofline fraction on the algorithmic bytes (own + other
features read once, output written once). A/B: TSPLAT_UV_COARSE_DIRECT=1 selects the
sample-then-dot kernel."""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from transplat_amd import _lib, kernels  # noqa: E402
from transplat_amd import synthetic as S  # noqa: E402
from transplat_amd.model.encoder.matching.depth_predictor_trans import prepare_feat_proj_data_lists  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--hw", type=int, default=64)
ap.add_argument("--iters", type=int, default=50)
args = ap.parse_args()
dev = torch.device("cuda:0")
_lib.load()
b, hw = args.batch, args.hw
ctx = S.make_batch(b, image_shape=(hw, hw))["context"]
_, intr, poses, disp = prepare_feat_proj_data_lists(torch.zeros((b, 2, 1, hw, hw)), ctx["intrinsics"],
                                                    ctx["extrinsics"], ctx["near"], ctx["far"], 128)
intr, pose, disp = intr.to(dev), poses[0].to(dev), disp.flatten(1).to(dev)
feat = torch.randn((b, 2, hw * hw, 128), device=dev)
for _ in range(3):
    kernels.uv_coarse(feat, intr, pose, disp, hw, hw)
torch.cuda.synchronize()
_lib.prof_enable("uv_coarse")
for _ in range(args.iters):
    kernels.uv_coarse(feat, intr, pose, disp, hw, hw)
ms, n = _lib.prof_read()
_lib.prof_enable(None)
us = ms / n * 1e3
nbytes = 2 * b * hw * hw * (128 * 4 * 2 + 128 * 4)
print(f"uv_coarse variant={'direct' if os.environ.get('TSPLAT_UV_COARSE_DIRECT') == '1' else 'dedup'} b={b} "
      f"hw={hw}: {us:.1f} us/call, {nbytes / us / 1e3:.1f} GB/s = {nbytes / us / 1e3 / 8000:.3f} of HBM peak", flush=True)
