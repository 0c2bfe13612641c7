"""DPT head 3x3 convolutions (the shapes the C2 step sends to MIOpen, tools/op_stacks.py): MIOpen on
the channels-last map (today's route) vs MIOpen NCHW vs the Winograd kernel on NCHW, and Winograd
with the two layout copies a channels-last caller would pay. Usage: python tools/bench_dpt_conv.py"""
import torch
import torch.nn.functional as F

from transplat_amd import kernels

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
SHAPES = [  # (n, ci, h, w, co), calls per C2 step
    ((2, 128, 9, 9, 128), 2), ((2, 128, 18, 18, 128), 4), ((2, 128, 36, 36, 128), 4),
    ((2, 128, 72, 72, 128), 4), ((2, 96, 72, 72, 128), 1), ((2, 192, 36, 36, 128), 1),
    ((2, 384, 18, 18, 128), 1), ((2, 768, 9, 9, 128), 1), ((2, 128, 144, 144, 64), 1),
    ((2, 64, 252, 252, 32), 1),
]


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / it


print(f"{'shape':28s} {'calls':>5s} {'miopen_cl':>9s} {'miopen':>8s} {'wino':>8s} {'wino+cp':>8s} {'err':>8s}")
tot = {"cl": 0.0, "nchw": 0.0, "wino": 0.0, "winocp": 0.0}
for (n, ci, h, w, co), calls in SHAPES:
    x = torch.randn(n, ci, h, w, device=dev)
    wt = torch.randn(co, ci, 3, 3, device=dev) / (3 * ci ** 0.5)
    xcl, wcl = x.to(memory_format=torch.channels_last), wt.to(memory_format=torch.channels_last)
    ok = kernels.conv3x3_wino_ok(x, wt, vs_miopen=True)
    t_cl = timeit(lambda: F.conv2d(xcl, wcl, padding=1))
    t_n = timeit(lambda: F.conv2d(x, wt, padding=1))
    t_w = timeit(lambda: kernels.conv3x3_wino(x, wt))
    t_wc = timeit(lambda: kernels.conv3x3_wino(xcl.contiguous(), wt).contiguous(memory_format=torch.channels_last))
    err = (kernels.conv3x3_wino(x, wt) - F.conv2d(x, wt, padding=1)).abs().max().item()
    for k, v in (("cl", t_cl), ("nchw", t_n), ("wino", t_w), ("winocp", t_wc)):
        tot[k] += v * calls
    print(f"{str((n, ci, h, w, co)):28s} {calls:5d} {t_cl:9.1f} {t_n:8.1f} {t_w:8.1f} {t_wc:8.1f} {err:8.1e}"
          f"{'' if ok else '  (rule: no)'}", flush=True)
print("per step (us):", {k: round(v, 1) for k, v in tot.items()})
