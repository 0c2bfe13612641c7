"""List the convolutions of one eager e2e step whose input is not NCHW-contiguous (channels-last
views from permute/rearrange make torch run the whole chain NHWC and re-layout weights per call).
usage: conv_layouts.py [--dense-dtype fp32]"""
import argparse

import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

ap = argparse.ArgumentParser()
ap.add_argument("--dense-dtype", default="fp32")
args = ap.parse_args()
dev = torch.device("cuda:0")
model = build_model(dev, args.dense_dtype)
names = {m: n for n, m in model.named_modules()}
seen = []


def _pre(mod, inp):
    x = inp[0]
    if isinstance(x, torch.Tensor) and not x.is_contiguous():
        cl = x.is_contiguous(memory_format=torch.channels_last) if x.dim() == 4 else False
        seen.append(f"{names[mod]:60s} {tuple(x.shape)} stride={x.stride()} channels_last={cl}")


for m in model.modules():
    if isinstance(m, (torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.ConvTranspose2d)):
        m.register_forward_pre_hook(_pre)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
with torch.no_grad():
    model.test_step(data)
torch.cuda.synchronize()
print(f"{len(seen)} convolutions with non-NCHW-contiguous input")
print("\n".join(seen))
