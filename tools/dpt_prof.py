"""The DPT head of the C2 step alone (DA-V2 ViT-B, 2 views at 252^2, bf16x3 mode): DINOv2 run once,
then head(features) captured in a hipGraph and replayed; prints the replay time. Under
rocprofv3 --kernel-trace --stats it gives the head's kernel mix. usage: dpt_prof.py [replays]"""
import sys

import torch

from transplat_amd import kernels as K
from transplat_amd.model.depth_anything.dpt import DepthAnythingV2

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = DepthAnythingV2(encoder="vitb", features=128, out_channels=[96, 192, 384, 768]).eval().to(dev)
K.install_linear_dispatch(m)
K.install_conv2d_dispatch(m)
x = torch.randn(2, 3, 252, 252, device=dev)
with torch.no_grad(), K.dense_precision("bf16x3"):
    head = m.depth_head
    head.prepare(True)
    feats = m.pretrained.get_intermediate_layers(x, m.intermediate_layer_idx["vitb"], return_class_token=True)
    for _ in range(2):
        head(feats, 18, 18)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        head(feats, 18, 18)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        g.replay()
    e.record()
    torch.cuda.synchronize()
print(f"DPT head replay: {s.elapsed_time(e) / n * 1e3:.1f} us", flush=True)
