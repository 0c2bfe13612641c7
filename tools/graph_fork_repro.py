"""Minimal hipGraph capture of nested stream forks (fork from a side stream onto a second side
stream, several times, then joins), to find out whether HIP's capture_end handles the pattern the
DPT branch hoisting produces. Usage: python tools/graph_fork_repro.py {nested,flat,nested_once}"""
import sys

import torch

mode = sys.argv[1]
dev = torch.device("cuda:0")
s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
x = torch.randn(1024, 1024, device=dev)


def body(x):
    main = torch.cuda.current_stream(dev)  # the capture stream inside torch.cuda.graph
    if mode == "flat":
        s0.wait_stream(main)
        with torch.cuda.stream(s0):
            a = x @ x
        s1.wait_stream(main)
        with torch.cuda.stream(s1):
            b = x + 1
        main.wait_stream(s0)
        main.wait_stream(s1)
        return a + b
    s0.wait_stream(main)
    with torch.cuda.stream(s0):
        h = x
        outs = []
        for k in range(3 if mode == "nested" else 1):
            h = h @ x
            s1.wait_stream(s0)
            with torch.cuda.stream(s1):
                outs.append(h * 2)
        h = h @ x
        for _ in outs:
            s0.wait_stream(s1)
        a = h + sum(outs)
    y = x * 3  # main's own work
    main.wait_stream(s0)
    return a + y


for _ in range(2):
    body(x)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = body(x)
g.replay()
torch.cuda.synchronize()
ref = body(x)
torch.cuda.synchronize()
print(mode, "ok", float((out - ref).abs().max()))
