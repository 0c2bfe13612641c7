"""Microbenchmark of the window-attention kernel alone (2-view 64x64 map, splits 2, C=128: the
transformer's shape at 256x256 input). Prints average µs per call (HIP events) and TFLOP/s.
Variants via env TSPLAT_WINATTN / TSPLAT_WINATTN_KSPLIT (see csrc/winattn.hip)."""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from transplat_amd import _lib, kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=2)
ap.add_argument("--hw", type=int, default=64)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--shift", type=int, default=1)
ap.add_argument("--dtype", choices=["fp32", "bf16", "x3"], default="fp32")
args = ap.parse_args()
dev = torch.device("cuda:0")
_lib.load()
b, hw = args.batch, args.hw
g = torch.Generator(device=dev).manual_seed(0)
dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
q, k, v = (torch.randn((b, hw * hw, 128), device=dev, generator=g).to(dt) for _ in range(3))
if args.dtype == "x3":  # bf16x3: K / V split once (as the merge path does per layer), main kernel timed
    L0 = (hw // 2) ** 2
    kv = kernels.split_kv_bf16x3(k, v)
    ws = torch.empty(max(int(_lib.load().tsplat_win_attn_workspace_bytes(b, hw, hw, 1, 2)), 4), dtype=torch.uint8,
                     device=dev)

    split = int(_lib.load().tsplat_win_attn_split(b, hw, hw, 1, 2))
    out = torch.empty_like(q)

    def attn():
        if split > 1:  # main kernel only (the merge projection folds the combine)
            _lib.check(_lib.load().tsplat_win_attn_x3_partials_fwd(_lib.ptr(q), _lib.ptr(kv), _lib.ptr(ws), b, hw, hw,
                                                                   128, 1, 2, int(args.shift), 0,
                                                                   _lib.stream_ptr(dev)), "x3")
        else:  # no key split: the kernel writes the normalised output
            _lib.check(_lib.load().tsplat_win_attn_x3_fwd(_lib.ptr(q), _lib.ptr(kv), _lib.ptr(out), _lib.ptr(ws), b, hw,
                                                          hw, 128, 1, 2, int(args.shift), _lib.stream_ptr(dev)), "x3")
else:
    def attn():
        kernels.window_attention(q, k, v, hw, hw, 2, bool(args.shift))
for _ in range(3):
    attn()
torch.cuda.synchronize()
_lib.prof_enable("win_attn")  # HIP events around the kernel launches only (no Python overhead)
for _ in range(args.iters):
    attn()
ms, n = _lib.prof_read()
_lib.prof_enable(None)
us = ms / n * 1e3
L = (hw // 2) ** 2
flops = 4 * b * 4 * L * L * 128
print(f"{args.dtype} variant={os.environ.get('TSPLAT_WINATTN', 'default')} ksplit={os.environ.get('TSPLAT_WINATTN_KSPLIT', 'auto')} "
      f"b={b} hw={hw}: {us:.1f} us/call, {flops / us / 1e6:.1f} TFLOP/s", flush=True)
