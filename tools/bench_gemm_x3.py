"""tsplat_gemm_x3_fwd alone on the DINOv2 shapes (M = 650 rows; slabs not summed), graph-timed.
usage: bench_gemm_x3.py [--m M]"""
import sys

import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
m = int(sys.argv[sys.argv.index("--m") + 1]) if "--m" in sys.argv else 650
K._DENSE = "bf16x3"
SHAPES = {"qkv": (768, 2304, "none"), "proj": (768, 768, "none"), "fc1": (768, 3072, "gelu"),
          "fc2": (3072, 768, "none"), "mvt_fc1": (256, 1024, "none")}


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


for name, (k, n, act) in SHAPES.items():
    mm = 8192 if name == "mvt_fc1" else m
    x = torch.randn(mm, k, device=dev)
    w = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev)
    line = []
    for s in ((1,) if act != "none" else (1, 2, 3, 4, 6, 8)):
        if s > 1 and (s - 1) * -(-(-(-k // 64)) // s) >= -(-k // 64):
            continue
        t = timeit(lambda: K.gemm_x3(x, w, b, act=act, ksplit=s))
        fl = 2 * mm * n * k * 3
        line.append(f"s{s} {t:5.1f}us ({fl / t / 1e6:5.0f} TF)")
    print(f"{name:8s} M={mm} K={k} N={n} auto=s{K.gemm_ksplit(mm, n, k)}: " + " | ".join(line), flush=True)
