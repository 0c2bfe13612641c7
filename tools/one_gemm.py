"""One tsplat_gemm_x3_fwd shape, launched `iters` times (for rocprofv3 counter passes).
usage: one_gemm.py M K N ksplit [act] [iters]"""
import sys

import torch

from transplat_amd import kernels as K

m, k, n, s = map(int, sys.argv[1:5])
act = sys.argv[5] if len(sys.argv) > 5 else "none"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda:0")
K._DENSE = "bf16x3"
x = torch.randn(m, k, device=dev)
w = torch.randn(n, k, device=dev) / k ** 0.5
b = torch.randn(n, device=dev)
for _ in range(iters):
    K.gemm_x3(x, w, b, act=act, ksplit=s)
torch.cuda.synchronize()
