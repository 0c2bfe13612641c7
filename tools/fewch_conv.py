"""Few-channel full-resolution 3x3 convolutions of the refine U-Net / heads (b = 1 shapes): the
bf16x3 Winograd vs the few-channel direct kernel (csrc/convfew.hip, where conv3x3_wino routes it) vs
the split-bf16 implicit-GEMM direct kernel, HIP-event averages of 50 calls after warmup."""
import torch

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
SHAPES = [(2, 32, 256, 256, 32), (2, 64, 256, 256, 32), (2, 38, 256, 256, 32), (2, 32, 256, 256, 64),
          (2, 64, 256, 256, 2), (2, 32, 128, 128, 32), (2, 64, 128, 128, 64), (2, 32, 64, 64, 32),
          (2, 128, 256, 256, 32), (16, 32, 256, 256, 32), (16, 64, 128, 128, 64)]


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


with K.dense_precision("bf16x3"):
    for n, ci, h, w, co in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev) * 0.05
        b = torch.randn(co, device=dev)
        ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), 1, 1).float()
        K._FEW = False
        yw = K.conv3x3_wino(x, wt, b)
        tw = timeit(lambda: K.conv3x3_wino(x, wt, b))
        K._FEW = True
        few = K._few_ok([x], n, h, w, co)
        yf = K.conv3x3_wino(x, wt, b)
        tf = timeit(lambda: K.conv3x3_wino(x, wt, b))
        yd = K.conv2d_direct(x, wt, b, 1)
        td = timeit(lambda: K.conv2d_direct(x, wt, b, 1))
        s = ref.abs().max().item()
        mb = (x.numel() + n * co * h * w) * 4 / 1e6
        print(f"{n}x{ci}->{co} @{h}x{w}: wino {tw:6.1f} us (err {(yw - ref).abs().max().item() / s:.1e})  "
              f"{'few' if few else 'route=wino'} {tf:6.1f} us (err {(yf - ref).abs().max().item() / s:.1e})  "
              f"direct {td:6.1f} us (err {(yd - ref).abs().max().item() / s:.1e})  I/O {mb:.1f} MB -> "
              f"{mb / 1e3 / (tf * 1e-6) / 1e3:.2f} TB/s on the routed one", flush=True)
