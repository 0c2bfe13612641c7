"""Attribute GPU time of one eager e2e step to PyTorch ops and their Python call sites
(torch.profiler), to find fusion targets.  usage: op_profile.py [--batch B] [--dense-dtype bf16]"""
import argparse
import collections

import torch
from torch.profiler import ProfilerActivity, profile

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--dense-dtype", default="fp32")
args = ap.parse_args()
dev = torch.device("cuda:0")
model = build_model(dev, args.dense_dtype)
data = S.make_batch(args.batch, image_shape=(256, 256), device=dev)
with torch.no_grad():
    for _ in range(3):
        model.test_step(data)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        model.test_step(data)
        torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=40,
                                                         max_shapes_column_width=80), flush=True)
# GPU time launched directly by each CPU op, by (op, innermost repo frame)
agg = collections.defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    dt = getattr(ev, "self_device_time_total", 0) or getattr(ev, "self_cuda_time_total", 0)
    if not dt or ev.device_type != torch.autograd.DeviceType.CPU:
        continue
    frames = [f for f in (ev.stack or []) if "transplat_amd" in f]
    where = frames[0].split("transplat_amd/")[-1] if frames else "?"
    a = agg[(ev.name, where)]
    a[0] += 1
    a[1] += dt
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
print("\n== GPU time by (op, call site)")
for (name, where), (n, us) in rows[:120]:
    print(f"{us:9.1f}us {n:4d}x {name[:34]:34s} {where}")
