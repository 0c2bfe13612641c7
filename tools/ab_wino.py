"""Same-process A/B of a Winograd-conv launch knob on the encoder's 3x3 shapes (tools/bench_wino.py's
census), graph-timed, alternating the settings per shape so clock drift hits both; prints per-shape
times, the call-weighted step total and each setting's max relative error against float64 conv2d.
usage: ab_wino.py [ENV_VAR] [VALUE_A] [VALUE_B]   (default: TSPLAT_WINO_WG 32 64)"""
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

VAR = sys.argv[1] if len(sys.argv) > 1 else "TSPLAT_WINO_WG"
MODES = tuple(sys.argv[2:4]) if len(sys.argv) > 3 else ("32", "64")
# the census list of tools/bench_wino.py (that script runs its benchmark at import)
src = Path(__file__).with_name("bench_wino.py").read_text()
SHAPES = eval(src.split("SHAPES = ", 1)[1].split("\n]\n", 1)[0] + "\n]")
dev = torch.device("cuda:0")


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * n) * 1e3


tot = {m: 0.0 for m in MODES}
print(f"{VAR}: {MODES[0]:>8s} {MODES[1]:>8s} (us)  calls  shape (n, ci, co, h, w)  rel.err")
with torch.no_grad():
    for (n, ci, co, h, w, calls) in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * (1.0 / (9 * ci) ** 0.5)
        b = torch.randn(co, device=dev)
        ref = F.conv2d(x.double(), wt.double(), b.double(), 1, 1)
        t, err = {}, {}
        for rep in range(2):
            for m in MODES:
                os.environ[VAR] = m
                tt = timeit(lambda: K.conv3x3_wino(x, wt, b))
                t[m] = min(t.get(m, 1e30), tt)
                if rep == 0:
                    err[m] = ((K.conv3x3_wino(x, wt, b).double() - ref).abs().max() / ref.abs().max()).item()
        for m in MODES:
            tot[m] += t[m] * calls
        print(f"{'':{len(VAR) + 1}s} {t[MODES[0]]:8.1f} {t[MODES[1]]:8.1f}  {calls:5d}  {(n, ci, co, h, w)}  "
              f"{err[MODES[0]]:.1e} / {err[MODES[1]]:.1e}", flush=True)
        assert max(err.values()) < 2e-5, err
print(f"total per step: {MODES[0]} {tot[MODES[0]]:.1f} us, {MODES[1]} {tot[MODES[1]]:.1f} us")
