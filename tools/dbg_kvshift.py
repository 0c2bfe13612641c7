"""Diagnostic: bf16 window attention with a key-batch shift vs rolled copies, and run-to-run
repeatability of each (max abs differences)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
from canonical import seeded  # noqa: E402
from transplat_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
for kern in ("v2", "v3"):
    os.environ["TSPLAT_WINATTN_BF16"] = kern
    for b, kvs in ((2, 1), (8, 4)):
        hw = 64
        q = seeded((b, hw * hw, 128), 97).bfloat16().to(dev)
        k = seeded((b, hw * hw, 128), 98).bfloat16().to(dev)
        v = seeded(k.shape, 99).bfloat16().to(dev)
        a1 = K.window_attention(q, k, v, hw, hw, 2, True, kv_shift=kvs)
        a2 = K.window_attention(q, k, v, hw, hw, 2, True, kv_shift=kvs)
        kr, vr = torch.roll(k, -kvs, dims=0), torch.roll(v, -kvs, dims=0)
        r1 = K.window_attention(q, kr, vr, hw, hw, 2, True)
        r2 = K.window_attention(q, kr, vr, hw, hw, 2, True)
        d = lambda x, y: (x.float() - y.float()).abs().max().item()
        print(f"{kern} b={b} s={kvs}: shift-vs-shift {d(a1, a2):.3e} roll-vs-roll {d(r1, r2):.3e} "
              f"shift-vs-roll {d(a1, r1):.3e} frac-differing {(a1 != r1).float().mean().item():.3e}", flush=True)
