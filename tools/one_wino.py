"""One Winograd convolution shape in a loop (for rocprofv3 PMC passes): n ci co h w [iters]."""
import sys

import torch

from transplat_amd import kernels as K

n, ci, co, h, w = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = torch.device("cuda:0")
x = torch.randn(n, ci, h, w, device=dev)
wt = torch.randn(co, ci, 3, 3, device=dev) * (1.0 / (9 * ci) ** 0.5)
for _ in range(iters):
    K.conv3x3_wino(x, wt)
torch.cuda.synchronize()
