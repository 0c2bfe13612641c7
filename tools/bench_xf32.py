"""hipBLASLt's emulated-xf32 fp32 GEMMs on gfx950 (the `S_MX_B` Tensile kernels: fp32 in / out,
F32XdlMathOp = bf16) vs its exact fp32 kernels on the C2 step's library GEMM shapes: time and max
error against float64 (relative to max |y|), next to a TF32-rounded emulation's error.
Mode from the environment: run once plain, once with HIPBLASLT_OVERRIDE_COMPUTE_TYPE_XF32=1, and
once with --allow-tf32 (torch.backends.cuda.matmul.allow_tf32 = True).
usage: [HIPBLASLT_OVERRIDE_COMPUTE_TYPE_XF32=1] bench_xf32.py [--allow-tf32]"""
import os
import sys

import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
if "--allow-tf32" in sys.argv:
    torch.backends.cuda.matmul.allow_tf32 = True
g = torch.Generator(device=dev).manual_seed(0)
mode = ("xf32-override " if os.environ.get("HIPBLASLT_OVERRIDE_COMPUTE_TYPE_XF32") else "") + (
    "allow_tf32" if "--allow-tf32" in sys.argv else "default")


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            fn()
    gr.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * n) * 1e3


def tf32(t):
    i = t.view(torch.int32)
    return ((i + 0xFFF + ((i >> 13) & 1)) & ~0x1FFF).view(torch.float32)


cases = [("dino qkv", 650, 768, 2304), ("dino proj", 650, 768, 768), ("dino fc1", 650, 768, 3072),
         ("dino fc2", 650, 3072, 768), ("mvt fc1", 8192, 256, 1024), ("mlp 128", 8192, 128, 512)]
print(f"mode: {mode}")
tot = 0.0
with torch.no_grad():
    for name, m, k, n in cases:
        x = torch.randn(m, k, device=dev, generator=g)
        w = torch.randn(n, k, device=dev, generator=g) / k ** 0.5
        b = torch.randn(n, device=dev, generator=g)
        ref = x.double() @ w.double().t() + b.double()
        sc = ref.abs().max().item()
        t = timeit(lambda: F.linear(x, w, b))
        e = ((F.linear(x, w, b).double() - ref).abs().max() / sc).item()
        etf = (((tf32(x).double() @ tf32(w).double().t() + b.double()) - ref).abs().max() / sc).item()
        # the same product without the bias epilogue: mm, and a 3-D matmul (bmm path)
        ref0 = x.double() @ w.double().t()
        sc0 = ref0.abs().max().item()
        wt = w.t()
        t_mm = timeit(lambda: torch.mm(x, wt))
        e_mm = ((torch.mm(x, wt).double() - ref0).abs().max() / sc0).item()
        x3 = x.unsqueeze(0)
        t_bmm = timeit(lambda: torch.matmul(x3, wt))
        e_bmm = ((torch.matmul(x3, wt)[0].double() - ref0).abs().max() / sc0).item()
        tot += t * (12 if name.startswith("dino") else 0)
        print(f"{name:10s} M={m:5d} K={k:5d} N={n:5d}: linear {t:6.1f} us ({2.0 * m * k * n / t / 1e6:6.1f} TF) "
              f"err {e:.1e} | mm {t_mm:6.1f} us err {e_mm:.1e} | matmul3d {t_bmm:6.1f} us err {e_bmm:.1e} "
              f"(tf32-emul {etf:.1e})", flush=True)
    a = torch.randn(2, 4096, 128, device=dev, generator=g)
    v = torch.randn(2, 4096, 128, device=dev, generator=g)
    ref = a.double() @ v.double().transpose(1, 2)
    t = timeit(lambda: torch.bmm(a, v.transpose(1, 2)))
    e = ((torch.bmm(a, v.transpose(1, 2)).double() - ref).abs().max() / ref.abs().max()).item()
    print(f"corr table 2x4096x4096x128: {t:7.1f} us  err {e:.1e}")
print(f"DINOv2 linears per step (x12): {tot:.1f} us")
