"""Time the depth predictor's dominant 3x3 convolutions under MIOpen: NCHW vs NHWC, fp32 vs bf16."""
import sys

import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = "--search" in sys.argv
shapes = [((2, 163, 256, 256), 168), ((2, 168, 256, 256), 84), ((2, 32, 256, 256), 32), ((2, 128, 64, 64), 128),
          ((2, 256, 64, 64), 128), ((2, 64, 256, 256), 32)]
for (n, c, h, w), co in shapes:
    for dt in (torch.float32, torch.bfloat16):
        for fmt in (torch.contiguous_format, torch.channels_last):
            x = torch.randn(n, c, h, w, device=dev, dtype=dt).to(memory_format=fmt)
            wt = torch.randn(co, c, 3, 3, device=dev, dtype=dt).to(memory_format=fmt)
            for _ in range(3):
                F.conv2d(x, wt, padding=1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                F.conv2d(x, wt, padding=1)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            fl = 2 * n * h * w * c * co * 9
            print(f"{str((n, c, h, w)):22s} -> {co:4d} {str(dt)[6:]:9s} {'NHWC' if fmt == torch.channels_last else 'NCHW'}: "
                  f"{us:8.1f} us  {fl / us / 1e6:6.1f} TFLOP/s", flush=True)
