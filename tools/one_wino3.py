"""One bf16x3 Winograd shape launched repeatedly (for rocprofv3 --pmc passes): n ci co h w [form]."""
import os
import sys

import torch

from transplat_amd import kernels as K

n, ci, co, h, w = (int(a) for a in sys.argv[1:6])
if len(sys.argv) > 6:
    os.environ["TSPLAT_WINO3_FORM"] = sys.argv[6]
dev = torch.device("cuda:0")
x = torch.randn(n, ci, h, w, device=dev)
wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
with torch.no_grad():
    for _ in range(10):
        K.conv3x3_wino(x, wt, None, precision="bf16x3")
torch.cuda.synchronize()
