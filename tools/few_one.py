"""One few-channel conv shape (csrc/convfew.hip) called N times (for rocprofv3 PMC / trace runs):
python tools/few_one.py n ci co h w [calls]"""
import sys

import torch

from transplat_amd import kernels as K

n, ci, co, h, w = (int(v) for v in sys.argv[1:6])
calls = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda:0")
x = torch.randn(n, ci, h, w, device=dev)
wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
b = torch.randn(co, device=dev)
with K.dense_precision("bf16x3"):
    assert K._few_ok([x], n, h, w, co)
    for _ in range(calls):
        K.conv3x3_wino(x, wt, b)
torch.cuda.synchronize()
