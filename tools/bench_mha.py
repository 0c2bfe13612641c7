"""DINOv2 attention at the C2 shape (2 images x 12 heads, 325 tokens, head dim 64): tsplat_mha_f32_fwd
vs torch SDPA on the same qkv, with the max deviation. Usage: python tools/bench_mha.py [--b 2]"""
import argparse

import torch
import torch.nn.functional as F

from transplat_amd import kernels

ap = argparse.ArgumentParser()
ap.add_argument("--b", type=int, default=2)
ap.add_argument("--iters", type=int, default=100)
args = ap.parse_args()
dev = torch.device("cuda:0")
B, N, H, D = args.b, 325, 12, 64
qkv = torch.randn(B, N, 3 * H * D, device=dev)
scale = D ** -0.5


def sdpa():
    q, k, v = qkv.view(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v, scale=scale).transpose(1, 2).reshape(B, N, H * D)


def timeit(fn):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / args.iters


flop = 4.0 * B * H * N * N * D
err = (kernels.mha(qkv, H, scale) - sdpa()).abs().max().item()
for name, fn in (("tsplat_mha_f32", lambda: kernels.mha(qkv, H, scale)), ("sdpa", sdpa)):
    t = timeit(fn)
    print(f"{name:16s} {t:7.1f} us  {flop / t / 1e6:6.1f} TFLOP/s", flush=True)
print(f"max |mha - sdpa| = {err:.2e}")
