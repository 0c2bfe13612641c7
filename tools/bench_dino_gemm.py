"""DINOv2 ViT-B linears at M = 650 rows (2 images x 325 tokens): F.linear exact fp32 vs the
emulated-xf32 library path vs split-K forms (K sliced over a batched GEMM, partials summed + bias),
graph-timed, each with its max error / max |y| against float64. usage: bench_dino_gemm.py"""
import sys

import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
torch.manual_seed(0)
M = 650
SHAPES = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}


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


def xf32(fn):
    def run():
        prev = torch.backends.cuda.matmul.allow_tf32
        torch.backends.cuda.matmul.allow_tf32 = True
        try:
            return fn()
        finally:
            torch.backends.cuda.matmul.allow_tf32 = prev
    return run


for name, (K, N) in SHAPES.items():
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    ref = F.linear(x.double(), w.double(), b.double())
    scale = ref.abs().max().item()
    forms = {"fp32": lambda: F.linear(x, w, b), "xf32": xf32(lambda: torch.matmul(x, w.t()) + b)}
    from transplat_amd import kernels as KK  # the hand-written split-bf16 GEMM (slabs summed for the error)
    KK._DENSE = "bf16x3"
    for s_ in (1, 2, 3, 4, 6, 8, 12):
        if s_ == 1 or (s_ <= K // 128):
            forms[f"gemm_x3_s{s_}"] = (lambda s_=s_: (lambda y: y if y.dim() == 2 else y.sum(0))(
                KK.gemm_x3(x, w, b, ksplit=s_)))
    forms["gemm_x3_auto"] = lambda: (lambda y: y if y.dim() == 2 else y.sum(0))(KK.gemm_x3(x, w, b, ksplit=0))
    if "--only-x3" in sys.argv:
        forms = {k_: v_ for k_, v_ in forms.items() if k_.startswith("gemm") or k_ == "fp32"}
    for s in (2, 4, 8):
        if K % s:
            continue
        xs = x.view(M, s, K // s).transpose(0, 1)           # [s, M, K/s] (strided view)
        ws = w.view(N, s, K // s).permute(1, 2, 0)          # [s, K/s, N]
        forms[f"splitK{s}"] = (lambda xs=xs, ws=ws: torch.bmm(xs, ws).sum(0) + b)
        forms[f"splitK{s}_xf32"] = xf32(lambda xs=xs, ws=ws: torch.bmm(xs, ws).sum(0) + b)
        xsc, wsc = xs.contiguous(), ws.contiguous()
        forms[f"splitK{s}c"] = (lambda xs=xsc, ws=wsc: torch.bmm(xs, ws).sum(0) + b)
    line = []
    for f, fn in forms.items():
        t = timeit(fn)
        err = (fn().double() - ref).abs().max().item() / scale
        line.append(f"{f} {t:6.1f}us ({err:.1e})")
    print(f"{name} K={K} N={N}: " + " | ".join(line), flush=True)
