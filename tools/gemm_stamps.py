"""Per-workgroup phase clocks of tsplat_gemm_x3_fwd (diagnostic build: tools/build_var.sh
tools/var/gemm_stamp.so gemm.hip -DTSPLAT_GEMM_STAMP=1; run with TSPLAT_LIB pointing at it).
Slots: 0 entry, 1 prologue done, 2-5 after chunks 0-3, 6 loop done, 7 end (100-MHz clock)."""
import ctypes

import torch

from transplat_amd import _lib
from transplat_amd import kernels as K

dev = torch.device("cuda:0")
K._DENSE = "bf16x3"
lib = _lib.load()
fn = lib.tsplat_gemm_stamps
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
buf = torch.zeros(1 << 14, 8, dtype=torch.int64, device=dev)


def q(t, f):
    t = t.float().sort().values
    return t[min(len(t) - 1, int(f * len(t)))].item() / 100.0


for (m, k, n, s, act) in [(650, 768, 3072, 1, "gelu"), (650, 768, 2304, 1, "none"), (650, 3072, 768, 6, "none"),
                          (650, 768, 768, 4, "none")]:
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev) / k ** 0.5
    for _ in range(3):
        K.gemm_x3(x, w, None, act=act, ksplit=s)
    torch.cuda.synchronize()
    buf.zero_()
    assert fn(buf.data_ptr()) == 0
    K.gemm_x3(x, w, None, act=act, ksplit=s)
    torch.cuda.synchronize()
    assert fn(None) == 0
    st = buf[buf[:, 0] != 0].cpu()
    t0 = st[:, 0].min()
    line = f"{(m, k, n, s)}: {len(st)} WGs span {(st[:, 7].max() - t0).item() / 100:6.2f} us, start max {(st[:, 0].max() - t0).item() / 100:5.2f}"
    for i, nm in enumerate(["prologue", "c0", "c1", "c2", "c3", "rest", "epilogue"]):
        a, b = (i, i + 1) if i < 5 else ((5, 6) if i == 5 else (6, 7))
        d = st[:, b] - st[:, a]
        ok = st[:, b] != 0
        if ok.any():
            line += f" | {nm} {q(d[ok], .5):5.2f}/{q(d[ok], .9):5.2f}"
    print(line, flush=True)
