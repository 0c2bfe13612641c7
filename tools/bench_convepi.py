"""conv + bias + act: module path (MIOpen conv with bias, PyTorch GELU) vs bias-free conv +
tsplat_bias_act_fwd, on the full-resolution Gaussian head shapes (b = 1, 2 views, 256x256)."""
import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
for cin, cout, act in [(163, 168, "gelu"), (168, 84, "none")]:
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(dev)
    x = torch.randn(2, cin, 256, 256, device=dev)
    a = lambda: F.gelu(conv(x)) if act == "gelu" else conv(x)
    b = lambda: K.conv_bias_act(conv, x, act)
    c = lambda: F.conv2d(x, conv.weight, None, 1, 1)
    for name, f in (("module", a), ("fused", b), ("conv-nobias", c)):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"{cin}->{cout} {act:5s} {name:12s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us", flush=True)
