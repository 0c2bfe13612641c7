"""Per-launch cost of a replayed hipGraph on this box: N dependent launches of a tiny elementwise
kernel captured into one graph (the C2 step is ~660 launches), timed with events over R replays.
usage: graph_launch_probe.py [N] [R]"""
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 660
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
x = torch.zeros(256, device="cuda")
for numel in (256, 1 << 20):
    x = torch.zeros(numel, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"graph of {n} dependent add_ launches on {numel} floats: {ms:.3f} ms per replay = "
          f"{ms / n * 1e3:.2f} us per launch", flush=True)
