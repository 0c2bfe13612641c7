"""Split-bf16 ("bf16x3") GEMMs on hipBLASLt vs exact fp32 for the C2 step's library GEMM shapes.

y = x W^T with x = xh + xl, W = Wh + Wl (bf16 halves) is taken as ONE bf16 GEMM with K' = 3K:
[xh | xh | xl] . [Wh | Wl | Wh]^T (the dropped xl Wl term and the halves' rounding leave ~2^-17
relative per product; TF32 rounds each operand to 2^-11). fp32 output via mm(out_dtype=fp32).
Prints per shape: fp32 F.linear time, the split GEMM time, the activation split time, and the
max error of both against float64 (relative to max |y|), next to a TF32-rounded emulation's.
"""
import torch
import torch.nn.functional as F

from transplat_amd import kernels as K

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def split3_act(x):
    xh = x.to(torch.bfloat16)
    xl = (x - xh.float()).to(torch.bfloat16)
    return torch.cat((xh, xh, xl), dim=-1)


def split3_w(w):
    wh = w.to(torch.bfloat16)
    wl = (w - wh.float()).to(torch.bfloat16)
    return torch.cat((wh, wl, wh), dim=-1)


def tf32(t):  # round to 10 explicit mantissa bits (nearest-even on the bits)
    i = t.view(torch.int32)
    r = ((i + 0xFFF + ((i >> 13) & 1)) & ~0x1FFF)
    return r.view(torch.float32)


cases = [("dino qkv", 650, 768, 2304), ("dino proj", 650, 768, 768), ("dino fc1", 650, 768, 3072),
         ("dino fc2", 650, 3072, 768), ("mvt fc1", 8192, 256, 1024), ("mlp0?", 8192, 128, 512)]
for name, m, k, n in cases:
    x = torch.randn(m, k, device=dev, generator=g)
    w = torch.randn(n, k, device=dev, generator=g) / k ** 0.5
    b = torch.randn(n, device=dev, generator=g)
    ref = (x.double() @ w.double().t() + b.double())
    scale = ref.abs().max().item()
    w3 = split3_w(w)
    x3 = split3_act(x)
    t_f32 = timeit(lambda: F.linear(x, w, b))
    t_s = timeit(lambda: torch.addmm(b, x3, w3.t(), out_dtype=torch.float32))
    t_split = timeit(lambda: split3_act(x))
    t_ours = timeit(lambda: K.linear_bf16x3(x, w, b))
    e_ours = ((K.linear_bf16x3(x, w, b).double() - ref).abs().max() / scale).item()
    y3 = torch.addmm(b, x3, w3.t(), out_dtype=torch.float32)
    e_f32 = ((F.linear(x, w, b).double() - ref).abs().max() / scale).item()
    e_s = ((y3.double() - ref).abs().max() / scale).item()
    e_tf = (((tf32(x).double() @ tf32(w).double().t() + b.double()) - ref).abs().max() / scale).item()
    fl = 2.0 * m * k * n
    print(f"{name:10s} M={m:5d} K={k:5d} N={n:5d}: fp32 {t_f32:7.1f} us ({fl / t_f32 / 1e6:6.1f} TF)  "
          f"bf16x3 gemm {t_s:7.1f} us  split(x) {t_split:6.1f} us  tsplat_linear_bf16x3 {t_ours:6.1f} us | "
          f"err fp32 {e_f32:.1e} bf16x3 {e_s:.1e} ours {e_ours:.1e} "
          f"tf32-emul {e_tf:.1e}", flush=True)

# correlation table: [2, 4096, 128] x [2, 128, 4096]
k_ = torch.randn(2, 4096, 128, device=dev, generator=g)
v_ = torch.randn(2, 4096, 128, device=dev, generator=g)
ref = k_.double() @ v_.double().transpose(1, 2)
scale = ref.abs().max().item()
k3, v3 = split3_act(k_), split3_w(v_)
t_f32 = timeit(lambda: torch.bmm(k_, v_.transpose(1, 2)))
t_s = timeit(lambda: torch.bmm(k3, v3.transpose(1, 2), out_dtype=torch.float32))
t_split = timeit(lambda: (split3_act(k_), split3_w(v_)))
e_s = ((torch.bmm(k3, v3.transpose(1, 2), out_dtype=torch.float32).double() - ref).abs().max() / scale).item()
e_f = ((torch.bmm(k_, v_.transpose(1, 2)).double() - ref).abs().max() / scale).item()
tab = torch.empty(2, 4096, 4096, device=dev)


def ours():
    for i in range(2):
        tab[i].copy_(K.linear_bf16x3(k_[i], v_[i], cache=False))


t_o = timeit(ours)
e_o = ((tab.double() - ref).abs().max() / scale).item()
print(f"corr table 2x4096x4096x128: fp32 {t_f32:.1f} us  bf16x3 {t_s:.1f} us  split {t_split:.1f} us  "
      f"tsplat_linear_bf16x3 x2 {t_o:.1f} us | err fp32 {e_f:.1e} bf16x3 {e_s:.1e} ours {e_o:.1e}", flush=True)
