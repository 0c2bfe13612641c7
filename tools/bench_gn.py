"""GroupNorm launch forms graph-timed: the two-launch stats + apply pair vs the one-launch
rendezvous form (tsplat_group_norm_sync_fwd), per shape. python tools/bench_gn.py"""
import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
SHAPES = [(2, 32, 256, 256, 32), (2, 64, 256, 256, 32), (2, 64, 128, 128, 32), (2, 128, 72, 72, 32),
          (2, 128, 144, 144, 32), (2, 32, 128, 128, 32)]


def timeit(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(20):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / 100


for n, c, h, w, groups in SHAPES:
    x = torch.randn(n, c, h, w, device=dev)
    wt, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    row = []
    for sync in (False, True):
        K._GN_SYNC = sync
        row.append(timeit(lambda: K.group_norm(x, groups, wt, b, 1e-5, "silu")))
    print(f"{(n, c, h, w, groups)}: two-launch {row[0]:6.1f} us  one-launch {row[1]:6.1f} us", flush=True)
