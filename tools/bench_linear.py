"""Microbenchmark of tsplat_linear_f32_fwd on the multi-view transformer's shapes at b = 1
(8,192 rows = 2 views x 64 x 64): HIP events around the launches, µs per call and TFLOP/s against
the 157.3 TF fp32-MFMA peak; next to torch's hipBLASLt F.linear for the plain GEMM part."""
import torch
import torch.nn.functional as F

from transplat_amd import _lib, kernels as K

dev = torch.device("cuda:0")
_lib.load()
g = torch.Generator(device=dev).manual_seed(0)
r = lambda *s: torch.randn(s, device=dev, generator=g)
M = 8192
cases = [  # name, k1, k2, n, kwargs
    ("qkv", 128, 0, 384, dict(split=True)),
    ("merge+ln+res", 128, 0, 128, dict(ln=True, res=True)),
    ("fc1+gelu [x|m]", 128, 128, 1024, dict(gelu=True)),
    ("fc2+ln+res", 1024, 0, 128, dict(ln=True, res=True)),
    ("gelu>fc2+ln+res", 1024, 0, 128, dict(ln=True, res=True, gelu_in=True)),
]
for name, k1, k2, n, kw in cases:
    x1, x2 = r(M, k1), (r(M, k2) if k2 else None)
    w = r(n, k1 + k2)
    ln = (r(n), r(n), 1e-5) if kw.get("ln") else None
    res = r(M, n) if kw.get("res") else None
    call = lambda: K.fused_linear(x1, w, x2=x2, gelu=kw.get("gelu", False), ln=ln, residual=res,
                                  split=kw.get("split", False), gelu_in=kw.get("gelu_in", False))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    _lib.prof_enable("linear")
    for _ in range(50):
        call()
    ms, cnt = _lib.prof_read()
    _lib.prof_enable(None)
    us = ms / cnt * 1e3
    xx = torch.cat([x1, x2], -1) if k2 else x1
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        F.linear(xx, w)
    e0.record()
    for _ in range(50):
        F.linear(xx, w)
    e1.record()
    torch.cuda.synchronize()
    tus = e0.elapsed_time(e1) / 50 * 1e3
    fl = 2.0 * M * (k1 + k2) * n
    print(f"{name:16s} M={M} K={k1 + k2} N={n}: fused {us:6.1f} us ({fl / us / 1e6:5.1f} TF, "
          f"{fl / us / 1e6 / 157.3 * 100:4.1f} %)   torch F.linear {tus:6.1f} us", flush=True)

# DINOv2 ViT-B (2 images x 325 tokens): qkv / proj / fc1 (+ exact GELU) / fc2, all with bias, vs
# hipBLASLt F.linear (+ F.gelu for fc1)
M = 650
for name, k, n, gelu in [("dino qkv", 768, 2304, False), ("dino proj", 768, 768, False),
                         ("dino fc1+gelu", 768, 3072, True), ("dino fc2", 3072, 768, False)]:
    x, w, bias = r(M, k), r(n, k), r(n)
    ours = lambda: K.fused_linear(x, w, bias=bias, gelu=gelu)
    ref = (lambda: F.gelu(F.linear(x, w, bias))) if gelu else (lambda: F.linear(x, w, bias))
    err = ((ours() - ref()).abs().max() / ref().abs().max()).item()
    ts = []
    for fn in (ours, ref):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 50 * 1e3)
    fl = 2.0 * M * k * n
    print(f"{name:16s} M={M} K={k} N={n}: fused {ts[0]:6.1f} us ({fl / ts[0] / 1e6:5.1f} TF)   "
          f"torch {ts[1]:6.1f} us ({fl / ts[1] / 1e6:5.1f} TF)  rel.err={err:.1e}", flush=True)
