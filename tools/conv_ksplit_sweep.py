"""Direct conv time vs waves per tile (ksplit) for a few U-Net shapes, graph-timed."""
import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * n) * 1e3


for (n, c, h, co) in [(2, 128, 16, 128), (2, 128, 32, 128), (2, 32, 16, 32), (2, 32, 128, 32)]:
    x = torch.randn(n, c, h, h, device=dev)
    w = torch.randn(co, c, 3, 3, device=dev)
    row = []
    for ks in (1, 2, 4, 8, 16):
        K._CONV_KSPLIT = ks
        row.append(f"ks{ks}={timeit(lambda: K.conv2d_direct(x, w)):.1f}")
    print((n, c, h, co), " ".join(row), flush=True)
K._CONV_KSPLIT = 0
x = torch.zeros(1, device=dev)
print(f"empty-ish launch (torch add): {timeit(lambda: x.add_(1)):.1f} us")
