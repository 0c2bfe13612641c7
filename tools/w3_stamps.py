"""Per-workgroup phase clocks of the bf16x3 Winograd kernels (diagnostic build tools/_bin/w3stamp.so,
tools/build_stamp_w3.sh; run with TSPLAT_LIB pointing at it). For each (shape, form): the launch's
span, the spread of workgroup start times, and the median / p90 of each phase, in us (100-MHz clock):
  conv_kernel:   0 entry, 1 prologue done (first region + A loads, first barrier), 2 loop done, 3 end
  persistent:    0 entry, 1 prologue done, 2 first block's loop done, 3 first block's epilogue done, 4 end
usage: TSPLAT_LIB=tools/_bin/w3stamp.so python tools/w3_stamps.py"""
import ctypes
import os

import torch

from transplat_amd import _lib
from transplat_amd import kernels as K

dev = torch.device("cuda:0")
CASES = [((2, 32, 32, 256, 256), "5"), ((2, 32, 32, 256, 256), "1"), ((2, 128, 128, 64, 64), "2"),
         ((2, 163, 168, 256, 256), "4"), ((2, 128, 32, 256, 256), "5")]

lib = _lib.load()
fn = lib.tsplat_wino3_stamps
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
buf = torch.zeros(1 << 16, 8, dtype=torch.int64, device=dev)


def q(t, f):
    t = t.float().sort().values
    return t[min(len(t) - 1, int(f * len(t)))].item() / 100.0  # 100 MHz ticks -> us


with torch.no_grad():
    for (n, ci, co, h, w), form in CASES:
        os.environ["TSPLAT_WINO3_FORM"] = form
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
        for _ in range(3):
            K.conv3x3_wino(x, wt, None, precision="bf16x3")
        torch.cuda.synchronize()
        buf.zero_()
        assert fn(buf.data_ptr()) == 0
        K.conv3x3_wino(x, wt, None, precision="bf16x3")
        torch.cuda.synchronize()
        assert fn(None) == 0
        st = buf[(buf[:, 0] != 0)].cpu()
        nslots = 5 if form == "5" else 4
        t0 = st[:, 0].min()
        span = (st[:, nslots - 1].max() - t0).item() / 100.0
        starts = st[:, 0] - t0
        line = (f"{(n, ci, co, h, w)} form {form}: {len(st)} WGs, span {span:6.1f} us, start p50/p90/max "
                f"{q(starts, .5):5.1f}/{q(starts, .9):5.1f}/{starts.max().item() / 100:5.1f}")
        names = ["prologue", "loop", "epilogue"] if nslots == 4 else ["prologue", "blk0 loop", "blk0 epi", "rest"]
        for i, nm in enumerate(names):
            d = st[:, i + 1] - st[:, i]
            line += f" | {nm} {q(d, .5):5.2f}/{q(d, .9):5.2f}"
        print(line, flush=True)
os.environ.pop("TSPLAT_WINO3_FORM", None)
