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
# module ranges, so every op can be attributed to the innermost module that launched it
_open = {}


def _pre(mod, *_):
    rf = torch.profiler.record_function("mod::" + type(mod).__name__)
    rf.__enter__()
    _open.setdefault(id(mod), []).append(rf)


def _post(mod, *_):
    _open[id(mod)].pop().__exit__(None, None, None)


for _m in model.modules():
    _m.register_forward_pre_hook(_pre)
    _m.register_forward_hook(_post)
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
    par, chain = ev.cpu_parent, []
    while par is not None and len(chain) < 2:
        if par.name.startswith("mod::"):
            chain.append(par.name[5:])
        par = par.cpu_parent
    where = "/".join(reversed(chain)) if chain else "?"
    a = agg[(ev.name, where)]
    a[0] += 1
    a[1] += dt
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
print("\n== GPU time by (op, call site)")
for (name, where), (n, us) in rows[:120]:
    print(f"{us:9.1f}us {n:4d}x {name[:34]:34s} {where}")
