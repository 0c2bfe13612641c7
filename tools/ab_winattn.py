"""Interleaved A/B timing of the window-attention entry point across several builds of the library
(same process, alternating rounds, HIP events around the C-ABI call; median per build).

    python tools/ab_winattn.py build/abl/lib0.so build/abl/libX.so --batch 2 --batch 16 [--dtype bf16]
Env knobs (TSPLAT_WINATTN...) apply to every build alike."""
import argparse
import ctypes

import torch

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--batch", type=int, action="append")
ap.add_argument("--hw", type=int, default=64)
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
ap.add_argument("--shift", type=int, default=1)
args = ap.parse_args()
dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
P, I, S = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
libs = []
for path in args.libs:
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    sfx = "_bf16" if args.dtype == "bf16" else ""
    fwd = getattr(lib, f"tsplat_win_attn{sfx}_fwd")
    fwd.argtypes = [P, P, P, P, P, I, I, I, I, I, I, I, P]
    fwd.restype = ctypes.c_int
    wsb = getattr(lib, f"tsplat_win_attn{sfx}_workspace_bytes")
    wsb.argtypes = [I, I, I, I, I]
    wsb.restype = S
    libs.append((path, fwd, wsb))
dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
stream = torch.cuda.current_stream(dev)
for b in args.batch or [2]:
    hw = args.hw
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v = (torch.randn((b, hw * hw, 128), device=dev, generator=g).to(dt) for _ in range(3))
    outs = []
    times = {p: [] for p, _, _ in libs}
    ref = None
    for rnd in range(args.rounds + 1):
        for path, fwd, wsb in libs:
            out = torch.empty_like(q)
            n = wsb(b, hw, hw, 1, 2)
            ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            call = lambda: fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), ws.data_ptr() if n else None,
                               b, hw, hw, 128, 1, 2, args.shift, stream.cuda_stream)
            assert call() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                call()
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                times[path].append(e0.elapsed_time(e1) / args.iters * 1e3)
            if rnd == args.rounds:
                if ref is None:
                    ref = out.float().clone()
                err = (out.float() - ref).abs().max().item()
                outs.append((path, err))
    L = (hw // 2) ** 2
    flops = 4 * b * 4 * L * L * 128
    for path, _, _ in libs:
        t = sorted(times[path])
        med = t[len(t) // 2]
        err = dict(outs)[path]
        print(f"{args.dtype} b={b}: {path:28s} median {med:7.1f} us  min {t[0]:7.1f}  {flops / med / 1e6:6.1f} TF/s  maxdiff-vs-first {err:.2e}",
              flush=True)
