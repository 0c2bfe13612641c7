"""Attribute GPU time of one e2e step to PyTorch ops (torch.profiler), to find fusion targets."""
import torch
from torch.profiler import ProfilerActivity, profile

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

dev = torch.device("cuda:0")
model = build_model(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
for _ in range(3):
    model.test_step(data)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    model.test_step(data)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=40,
                                                         max_shapes_column_width=70))
print(prof.key_averages(group_by_stack_n=6).table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=40))
