"""Segment shares of the key-pair window-attention loop from a TSPLAT_WA_STAMP diagnostic build.

    bash tools/build_ablation.sh && (stamp build: see tools/stamp_build.sh)
    TSPLAT_LIB=build/abl/lib_stamp.so TSPLAT_WINATTN=pair TSPLAT_WINATTN_KSPLIT=2 python tools/diag_wa_stamps.py --batch 16

Per-wave s_memtime sums (100 MHz... counted in s_memtime units) per segment, averaged over waves."""
import argparse
import ctypes

import numpy as np
import torch

from transplat_amd import _lib, kernels

SEGS = ["prologue", "QK issue", "mask+softmax", "barrier1", "storeK+loadV", "PV issue", "barrier2",
        "storeV", "merge", "-"]
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=2)
ap.add_argument("--hw", type=int, default=64)
args = ap.parse_args()
dev = torch.device("cuda:0")
lib = _lib.load()
b, hw = args.batch, args.hw
g = torch.Generator(device=dev).manual_seed(0)
q, k, v = (torch.randn((b, hw * hw, 128), device=dev, generator=g) for _ in range(3))
for _ in range(3):
    kernels.window_attention(q, k, v, hw, hw, 2, True)
torch.cuda.synchronize()
n = 8192
buf = np.zeros((n, 10), dtype=np.uint64)
fn = lib.tsplat_diag_wa_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
got = fn(buf.ctypes.data, n)
rows = buf[: got][buf[:got].sum(1) > 0].astype(np.float64)
print(f"b={b}: {len(rows)} waves stamped")
tot = rows.sum(1).mean()
for i, name in enumerate(SEGS[:9]):
    m = rows[:, i].mean()
    print(f"  {name:14s} {m:10.0f}  {100 * m / tot:5.1f}%")
print(f"  total          {tot:10.0f}")
