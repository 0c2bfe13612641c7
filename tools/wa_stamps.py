"""Per-workgroup phase clocks of the fp32 x32 window-attention kernel (diagnostic build
tools/_bin/wastamp.so, tools/build_stamp_wa.sh; run with TSPLAT_LIB pointing at it).
For each shape: workgroups per CU (HW_ID / XCC_ID), the spread of start times, the shader clock
rate, and the median / p90 of each phase in shader cycles: prologue (Q + first K/V tile, first
barrier), each key tile, epilogue (partial or output store).
usage: TSPLAT_LIB=tools/_bin/wastamp.so python tools/wa_stamps.py [--x3 | --bf16]  (--x3: the bf16x3 kernel,
--bf16: bf16 operands, i.e. the v3 kernel at b = 16 -- there "tile t" is the MFMA interval of tile t)"""
import collections
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from transplat_amd import _lib, kernels  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
fn = lib.tsplat_win_attn_stamps
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
buf = torch.zeros(1 << 14, 16, dtype=torch.int64, device=dev)


def q(t, f):
    t = t.double().sort().values
    return t[min(len(t) - 1, int(f * len(t)))].item()


X3 = "--x3" in sys.argv
BF16 = "--bf16" in sys.argv  # the bf16 v3 kernel (B >= 8 windows x 4 query blocks: b = 16 here)
attn = kernels.window_attention_x3 if X3 else kernels.window_attention
g = torch.Generator(device=dev).manual_seed(0)
with torch.no_grad():
    for b, shift in ((2, 0), (2, 1), (16, 1)):
        hw = 64
        qq, k, v = (torch.randn((b, hw * hw, 128), device=dev, generator=g) for _ in range(3))
        if BF16:
            qq, k, v = qq.bfloat16(), k.bfloat16(), v.bfloat16()
        for _ in range(3):
            attn(qq, k, v, hw, hw, 2, bool(shift))
        torch.cuda.synchronize()
        buf.zero_()
        assert fn(buf.data_ptr()) == 0
        attn(qq, k, v, hw, hw, 2, bool(shift))
        torch.cuda.synchronize()
        assert fn(None) == 0
        st = buf[buf[:, 0] != 0].cpu()
        n = len(st)
        if n == 0:
            print(f"b={b} shift={shift}: no stamps (a kernel form without phase clocks)", flush=True)
            continue
        hwid = st[:, 1]
        cu_key = ((hwid >> 32) & 0xF) * 256 + ((hwid >> 8) & 0xFF)  # xcc, (se, sh, cu)
        per_cu = collections.Counter(cu_key.tolist())
        hist = collections.Counter(per_cu.values())
        t0 = st[:, 0].min()
        span = (st[:, 13].max() - t0).item() / 100.0
        starts = (st[:, 0] - t0).double() / 100.0
        wall = (st[:, 13] - st[:, 0]).double() / 100.0
        cyc = (st[:, 12] - st[:, 2]).double()
        ghz = q(cyc / (wall * 1e3), 0.5)
        tiles = [i for i in range(8) if (st[:, 4 + i] != 0).all()]
        print(f"b={b} shift={shift}: {n} WGs on {len(per_cu)} CUs (WGs per CU: {dict(sorted(hist.items()))}), "
              f"span {span:.1f} us, start p50/p90/max {q(starts, .5):.1f}/{q(starts, .9):.1f}/{starts.max():.1f} us, "
              f"WG wall p50/p90/max {q(wall, .5):.1f}/{q(wall, .9):.1f}/{wall.max():.1f} us, clock {ghz:.2f} GHz", flush=True)
        ph = [("prologue", st[:, 3] - st[:, 2])]
        prev = st[:, 3]
        for i in tiles:
            ph.append((f"tile{i}", st[:, 4 + i] - prev))
            prev = st[:, 4 + i]
        ph.append(("epilogue", st[:, 12] - prev))
        print("   cycles p50/p90: " + " | ".join(f"{nm} {q(d, .5):.0f}/{q(d, .9):.0f}" for nm, d in ph), flush=True)
        # workgroups that shared a CU with another one vs alone
        shared = torch.tensor([per_cu[x] > 1 for x in cu_key.tolist()])
        if shared.any() and (~shared).any():
            print(f"   WG wall alone p50 {q(wall[~shared], .5):.1f} us vs sharing a CU p50 {q(wall[shared], .5):.1f} us "
                  f"({int(shared.sum())} WGs share)", flush=True)
