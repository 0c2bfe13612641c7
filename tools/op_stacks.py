"""Which Python call sites launch the small copy / add kernels of one e2e step (torch.profiler stacks)."""
import collections

import torch
from torch.profiler import ProfilerActivity, profile

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

dev = torch.device("cuda:0")
model = build_model(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
for _ in range(2):
    model.test_step(data)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    model.test_step(data)
    torch.cuda.synchronize()
agg = collections.Counter()
shown = False
for ev in prof.events():
    if not shown and ev.name == "aten::copy_":
        print("sample stack:", ev.stack[:8] if ev.stack else ev.stack)
        shown = True
    if ev.name in ("aten::copy_", "aten::add_", "aten::add", "aten::mul", "aten::cat", "aten::fill_", "aten::div"):
        frames = [f for f in (ev.stack or []) if "transplat_amd" in f or "repo/" in f]
        where = frames[0] if frames else "?"
        agg[(ev.name, where)] += 1
for (name, where), n in agg.most_common(40):
    print(f"{n:4d} {name:12s} {where}")
