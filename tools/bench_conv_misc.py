"""Which C3 convolutions still run as MIOpen im2col + GEMM per image: time the candidates under bf16
autocast and in fp32. Usage: python tools/bench_conv_misc.py"""
import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
CASES = [  # x shape, w shape, stride, padding
    ((16, 3, 256, 256), (64, 3, 7, 7), 2, 3),
    ((16, 64, 128, 128), (96, 64, 3, 3), 2, 1),
    ((16, 64, 128, 128), (96, 64, 1, 1), 2, 0),
    ((8, 128, 64, 64), (128, 128, 3, 3), 1, 1),
    ((16, 3, 252, 252), (768, 3, 14, 14), 14, 0),
]


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for xs, ws, st, pad in CASES:
    x = torch.randn(xs, device=dev)
    w = torch.randn(ws, device=dev) * 0.05
    with torch.no_grad():
        f32 = timed(lambda: F.conv2d(x, w, None, st, pad))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            bf = timed(lambda: F.conv2d(x, w, None, st, pad))
    print(f"x{xs} w{ws} s{st}: fp32 {f32:8.1f} us  autocast-bf16 {bf:8.1f} us", flush=True)
