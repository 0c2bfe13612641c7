"""One bf16 implicit-GEMM convolution shape run a few times (for rocprofv3 PMC passes over the kernel):
default 16 x 128 -> 128 at 64^2, 3x3 (the register-blocked form, C3's U-Net levels).
Usage: python tools/one_convbf16.py [n ci h w co] [--iters 10]"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from transplat_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("shape", nargs="*", type=int, default=[16, 128, 64, 64, 128])
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
n, ci, h, w, co = a.shape
dev = torch.device("cuda:0")
x = torch.randn(n, ci, h, w, device=dev).to(torch.bfloat16)
wt = (torch.randn(co, ci, 3, 3, device=dev) / (9 * ci) ** 0.5).to(torch.bfloat16)
b = torch.randn(co, device=dev).to(torch.bfloat16)
for _ in range(a.iters):
    y = K.conv_bf16(x, wt, b)
torch.cuda.synchronize()
print("ok", tuple(y.shape), y.dtype)
