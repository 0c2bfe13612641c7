"""Direct fp32 MFMA convolution of the U-Nets' low-resolution levels (tsplat_conv2d_f32_fwd via
kernels.conv2d_direct) against the oracle restatement (torch fp32 conv2d of the concatenated /
nearest-upsampled input, on the CPU).

Tolerance: exact fp32 products, different summation order over cin * k * k <= 2304 terms:
2e-5 of the output's max magnitude."""
import sys
from pathlib import Path

import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
from canonical import seeded  # noqa: E402

from oracle import encoder_ops as E  # noqa: E402

@pytest.fixture(autouse=True)
def _winograd_tests_run_winograd(request, monkeypatch):
    """The Winograd tests below pin the Winograd kernel; conv3x3_wino routes few-channel full-resolution
    shapes to the direct kernel of csrc/convfew.hip instead (tested by the *few* tests)."""
    if "wino" in request.node.name and "few" not in request.node.name:
        from transplat_amd import kernels as K

        monkeypatch.setattr(K, "_FEW", False)


CASES = [
    # n, c1, c2, h, w, cout, k, stride, upsample, bias
    (2, 32, 0, 16, 16, 32, 3, 1, False, False),
    (2, 128, 0, 16, 16, 128, 3, 1, False, True),
    (2, 128, 128, 16, 16, 128, 3, 1, False, False),   # output-block ResBlock on cat([h, skip])
    (2, 128, 128, 32, 32, 128, 1, 1, False, True),    # its 1x1 skip convolution
    (2, 32, 0, 32, 32, 32, 3, 2, False, True),        # Downsample
    (2, 128, 0, 16, 16, 128, 3, 1, True, True),       # Upsample (nearest 2x -> conv)
    (2, 32, 32, 64, 64, 32, 3, 1, False, False),
    (1, 6, 4, 9, 13, 40, 3, 1, False, True),          # ragged: odd sizes, cout % 32 != 0, tiny cin
    (1, 6, 0, 9, 13, 40, 3, 2, False, True),
    (3, 2, 0, 5, 7, 1, 3, 1, True, True),
    (2, 128, 0, 32, 32, 128, 3, 2, False, True),      # single-shot (4 ci pairs per wave) stride 2
    (2, 64, 0, 128, 128, 96, 1, 2, False, True),      # the UniMatch CNN's strided 1x1 shortcut
    (1, 6, 0, 9, 13, 40, 1, 2, False, False),         # strided 1x1, ragged
    (1, 96, 0, 12, 12, 64, 3, 1, False, True),        # single-shot with 3 pairs per wave
]


def test_oracle_conv2d_direct_matches_cat_and_interpolate():
    x1, x2 = seeded((1, 4, 6, 6), 1), seeded((1, 2, 6, 6), 2)
    w, b = seeded((5, 6, 3, 3), 3), seeded((5,), 4)
    ref = torch.nn.functional.conv2d(torch.nn.functional.interpolate(torch.cat([x1, x2], 1), scale_factor=2), w, b,
                                     padding=1)
    torch.testing.assert_close(E.conv2d_direct(x1, w, b, 1, x2=x2, upsample=True), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [3, 1])
def test_conv2d_direct_nonfinite_corner(device, k):
    """Zero-padding semantics with a non-finite input: an Inf at pixel (0, 0) reaches exactly the
    outputs whose receptive field holds it (as torch's conv2d); the kernel's masked padding taps
    (clamped loads of that same pixel) contribute +0, not Inf * 0 = NaN, everywhere else."""
    from transplat_amd import kernels as K

    x = seeded((1, 32, 16, 16), 21)
    x[0, 3, 0, 0] = float("inf")
    wt = seeded((32, 32, k, k), 22) * (1.0 / 32**0.5)
    ref = E.conv2d_direct(x, wt, None, 1)
    out = K.conv2d_direct(x.to(device), wt.to(device), None, 1).cpu()
    fin = torch.isfinite(ref)
    assert (~fin).any() and fin.any()
    assert torch.equal(torch.isfinite(out), fin)
    err = (out[fin] - ref[fin]).abs().max().item() / ref[fin].abs().max().item()
    assert err < 2e-5, err


@pytest.mark.gpu
@pytest.mark.parametrize("n,c1,c2,h,w,cout,k,stride,up,has_bias", CASES)
def test_conv2d_direct_kernel(device, n, c1, c2, h, w, cout, k, stride, up, has_bias):
    from transplat_amd import kernels as K

    x1 = seeded((n, c1, h, w), 11)
    x2 = seeded((n, c2, h, w), 12) if c2 else None
    wt = seeded((cout, c1 + c2, k, k), 13) * (1.0 / (c1 + c2) ** 0.5)
    b = seeded((cout,), 14) if has_bias else None
    ref = E.conv2d_direct(x1, wt, b, stride, x2=x2, upsample=up)
    out = K.conv2d_direct(x1.to(device), wt.to(device), b.to(device) if b is not None else None, stride,
                          x2=x2.to(device) if x2 is not None else None, upsample=up).cpu()
    assert out.shape == ref.shape
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err


@pytest.mark.gpu
@pytest.mark.parametrize("n,ci,h,w,co,k,stride,zmax", [(2, 768, 9, 9, 128, 3, 1, 64), (2, 256, 16, 16, 128, 3, 1, 64),
                                                      (2, 384, 18, 18, 128, 3, 1, 64), (1, 768, 9, 9, 96, 1, 1, 64),
                                                      (2, 768, 18, 18, 64, 3, 2, 4), (2, 512, 5, 7, 40, 3, 1, 3)])
def test_conv2d_direct_zsplit(device, monkeypatch, n, ci, h, w, co, k, stride, zmax):
    """tsplat_conv2d_f32_zsplit_fwd (ci pairs of each tile over zsplit workgroups, the last arriving
    one sums the partials in z order): against the oracle at the direct kernel's 2e-5; bit-identical
    over repeated launches (the counters reset themselves, the sum order does not depend on arrival
    order); ragged tiles and a non-power-of-2 cap (zmax 3 -> zsplit 2)."""
    from transplat_amd import kernels as K

    monkeypatch.setattr(K, "_ZSPLIT", zmax)
    x = seeded((n, ci, h, w), 31)
    wt = seeded((co, ci, k, k), 32) * (1.0 / ci**0.5)
    b = seeded((co,), 33)
    ho = (h + 2 * (k // 2) - k) // stride + 1
    wo = (w + 2 * (k // 2) - k) // stride + 1
    tiles = -(-(n * ho * wo) // 32) * -(-co // 32)
    assert K.conv_zsplit(tiles, ci // 2, 16, k) > 1
    ref = E.conv2d_direct(x, wt, b, stride)
    xd, wd, bd = x.to(device), wt.to(device), b.to(device)
    outs = [K.conv2d_direct(xd, wd, bd, stride).cpu() for _ in range(3)]
    err = (outs[0] - ref).abs().max().item() / ref.abs().max().item()
    print(f"zsplit {(n, ci, h, w, co, k, stride)}: z = {K.conv_zsplit(tiles, ci // 2, 16, k)}, rel err {err:.2e}")
    assert err < 2e-5, err
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    monkeypatch.setattr(K, "_ZSPLIT", 0)
    one = K.conv2d_direct(xd, wd, bd, stride).cpu()
    assert (one - ref).abs().max().item() / ref.abs().max().item() < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("n,ci,co,h,w,s", [(2, 96, 96, 18, 18, 4), (2, 192, 192, 18, 18, 2), (1, 6, 10, 5, 7, 3)])
def test_conv_transpose_direct(device, n, ci, co, h, w, s):
    """ConvTranspose2d with kernel = stride (the DPT's resize_layers, reference dpt.py:105-118) as a
    1x1 convolution to co s^2 channels on the direct exact-fp32 kernel + pixel_shuffle, vs float64."""
    from transplat_amd import kernels as K

    x = seeded((n, ci, h, w), 71)
    wt = seeded((ci, co, s, s), 72) / ci ** 0.5
    b = seeded((co,), 73)
    ref = torch.nn.functional.conv_transpose2d(x.double(), wt.double(), b.double(), stride=s)
    out = K.conv_transpose_direct(x.to(device), wt.to(device), b.to(device), s).cpu().double()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    m = torch.nn.ConvTranspose2d(ci, co, s, stride=s).to(device)
    K.install_conv2d_dispatch(m)
    with torch.no_grad():
        m.weight.copy_(wt.to(device))
        m.bias.copy_(b.to(device))
        assert torch.equal(m(x.to(device)), K.conv_transpose_direct(x.to(device), m.weight, m.bias, s))


@pytest.mark.gpu
@pytest.mark.parametrize("bias", [False, True])
def test_conv_unfold_gemm_stem(device, bias):
    """The UniMatch CNN's 7x7 stride-2 stem on 3 channels as im2col + one exact-fp32 GEMM per image
    (bias in the GEMM), vs float64, and through the installed Conv2d dispatch."""
    from transplat_amd import kernels as K

    x = seeded((2, 3, 256, 256), 74)
    wt = seeded((64, 3, 7, 7), 75) / 147 ** 0.5
    b = seeded((64,), 76) if bias else None
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double() if bias else None, stride=2, padding=3)
    out = K.conv_unfold_gemm(x.to(device), wt.to(device), b.to(device) if bias else None, 2, 3).cpu().double()
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    m = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(device)
    K.install_conv2d_dispatch(m)
    with torch.no_grad():
        m.weight.copy_(wt.to(device))
        assert torch.equal(m(x.to(device)), K.conv_unfold_gemm(x.to(device), m.weight, None, 2, 3))


@pytest.mark.gpu
def test_encoder_runs_no_library_convolution(device):
    """In the bench's default dense mode (bf16x3) every convolution of the encoder's step (UniMatch
    CNN, camera encoder, DA-V2's DPT head, U-Nets, heads) runs on the hand-written kernels: no aten
    convolution reaches MIOpen, so no algorithm choice by timing (cudnn.benchmark) can change the
    step's bits from one process to the next. (The exact-fp32 mode keeps the DPT head's
    channels-last 3x3s on MIOpen's NHWC kernels.)"""
    dense = "bf16x3"
    import sys
    from pathlib import Path

    from torch.utils._python_dispatch import TorchDispatchMode

    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    from canonical import canonical_init

    from transplat_amd import synthetic as S
    from transplat_amd.model.encoder import EncoderTrans, EncoderTransCfg

    class Convs(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.seen = []

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if "convolution" in func.__name__:
                self.seen.append((func.__name__, tuple(args[0].shape), tuple(args[1].shape)))
            return func(*args, **(kwargs or {}))

    enc = canonical_init(EncoderTrans(EncoderTransCfg(dense_dtype=dense)), seed=61).eval().to(device)
    ctx = {k: t.to(device) for k, t in S.make_batch(1, image_shape=(256, 256))["context"].items()}
    mode = Convs()
    with torch.no_grad(), mode:
        enc(ctx, global_step=0, deterministic=True)
    assert not mode.seen, mode.seen


@pytest.mark.gpu
def test_conv2d_direct_weight_cache_tracks_updates(device):
    """The packed-weight cache is keyed on the tensor version: an in-place update repacks."""
    from transplat_amd import kernels as K

    x = seeded((1, 32, 16, 16), 21).to(device)
    wt = seeded((32, 32, 3, 3), 22).to(device)
    y0 = K.conv2d_direct(x, wt)
    wt.mul_(2.0)
    y1 = K.conv2d_direct(x, wt)
    torch.testing.assert_close(y1, 2 * y0, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,h,w,cout,k,relu,res,bias", [
    (2, 128, 9, 9, 128, 3, True, False, True), (2, 128, 18, 18, 128, 3, True, True, True),
    (2, 128, 36, 36, 128, 3, False, True, False), (2, 128, 18, 18, 128, 1, False, False, True),
    (1, 6, 5, 7, 40, 3, True, True, True)])
def test_conv2d_nhwc_kernel(device, n, c, h, w, cout, k, relu, res, bias):
    """Channels-last variant (DPT ResidualConvUnit: ReLU on load, bias, residual) vs the oracle."""
    from transplat_amd import kernels as K

    x = seeded((n, c, h, w), 31)
    wt = seeded((cout, c, k, k), 32) * (1.0 / c ** 0.5)
    b = seeded((cout,), 33) if bias else None
    r = seeded((n, cout, h, w), 34) if res else None
    ref = E.conv2d_nhwc(x, wt, b, residual=r, relu_in=relu)
    cl = lambda t: t.to(device).contiguous(memory_format=torch.channels_last)  # noqa: E731
    assert K.conv2d_nhwc_ok(cl(x), wt.to(device)) or c < 8
    out = K.conv2d_nhwc(cl(x), wt.to(device), b.to(device) if b is not None else None,
                        residual=cl(r) if r is not None else None, relu_in=relu)
    assert out.is_contiguous(memory_format=torch.channels_last)
    err = (out.cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err


@pytest.mark.gpu
def test_conv1d_k1_through_direct_kernel(device):
    """The U-Net attention blocks' Conv1d(k=1) (qkv, proj_out) run as the 1x1 direct conv on [n, c, t, 1]."""
    from transplat_amd import kernels as K

    x = seeded((2, 128, 256), 41)
    wt, b = seeded((384, 128, 1), 42) * 0.1, seeded((384,), 43)
    ref = torch.nn.functional.conv1d(x, wt, b)
    xd = x.to(device).unsqueeze(-1)
    assert K.conv2d_direct_ok(xd, wt.to(device))
    out = K.conv2d_direct(xd, wt.to(device), b.to(device)).squeeze(-1).cpu()
    assert (out - ref).abs().max().item() < 2e-5 * ref.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("act,nres", [("relu", 0), ("none", 1), ("none", 2), ("gelu", 1)])
def test_conv_nhwc_epilogue(device, act, nres):
    """Bias-free MIOpen conv on channels-last maps + tsplat_bias_act_nhwc_fwd (bias, act, residuals)
    vs the module chain (DPT ResidualConvUnit / FeatureFusionBlock)."""
    from transplat_amd import kernels as K

    torch.manual_seed(0)
    conv = torch.nn.Conv2d(128, 128, 3, padding=1)
    x = seeded((2, 128, 18, 18), 51)
    rs = [seeded((2, 128, 18, 18), 52 + i) for i in range(nres)] + [None] * (2 - nres)
    with torch.no_grad():
        ref = E.conv_nhwc_epilogue(conv, x, act, *rs)
        cd = conv.to(device)
        cd.weight.data = cd.weight.data.contiguous(memory_format=torch.channels_last)
        cl = lambda t: t.to(device).contiguous(memory_format=torch.channels_last) if t is not None else None  # noqa
        out = K.conv_nhwc_epilogue(cd, cl(x), act, *[cl(r) for r in rs])
    assert out.is_contiguous(memory_format=torch.channels_last)
    err = (out.cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


@pytest.mark.gpu
def test_patch_embed_gemm_matches_conv(device):
    """DINOv2 PatchEmbed's fp32 device path (unfold + one GEMM) vs the stride-14 convolution."""
    from transplat_amd.model.depth_anything.dinov2 import PatchEmbed

    torch.manual_seed(0)
    pe = PatchEmbed(img_size=252, patch_size=14, in_chans=3, embed_dim=768)
    x = seeded((2, 3, 252, 252), 61)
    with torch.no_grad():
        ref = pe.proj(x).flatten(2).transpose(1, 2)
        out = pe.to(device)(x.to(device)).cpu()
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() < 2e-5 * ref.abs().max().item()


@pytest.mark.gpu
def test_unet_full_res_1x1_gemm_path(device, monkeypatch):
    """The U-Net's 1x1 convolutions that the direct kernel does not take run as a batched GEMM
    (ldm_unet.conv): same result as the convolution, with and without bias."""
    from transplat_amd import kernels as K
    from transplat_amd.model.encoder.matching import ldm_unet as U

    monkeypatch.setattr(K, "_CONV_MODE", "off")
    x = seeded((2, 64, 64, 64), 71)
    for bias in (True, False):
        torch.manual_seed(0)
        conv = torch.nn.Conv2d(64, 32, 1, bias=bias)
        with torch.no_grad():
            ref = conv(x)
            out = U.conv(conv.to(device), x.to(device)).cpu()
        assert (out - ref).abs().max().item() < 2e-5 * ref.abs().max().item()


WINO_CASES = [
    # n, ci, co, h, w, bias, act
    (2, 163, 168, 32, 32, True, "gelu"),   # to_gaussians' shape class: ci % 8 != 0, co % 32 != 0
    (2, 168, 84, 16, 40, True, "none"),    # to_disparity-like, tile rows of 20 (tbx 16)
    (2, 32, 32, 64, 64, False, "relu"),
    (1, 38, 32, 17, 21, True, "none"),     # odd sizes: half tiles on the last row / column (tbx 8)
    (1, 128, 128, 18, 18, True, "gelu"),   # tw 9 -> tbx 8
    (3, 16, 16, 9, 70, False, "none"),     # tw 35 -> tbx 32, a partial second tile block per row
    (1, 64, 2, 40, 36, True, "none"),      # a 2-channel head (co << 32: one mostly idle output block)
]


@pytest.mark.gpu
@pytest.mark.parametrize("wg", ["auto", "32", "32x2", "64"])
@pytest.mark.parametrize("n,ci,co,h,w,bias,act", WINO_CASES)
def test_conv3x3_wino_kernel(device, monkeypatch, wg, n, ci, co, h, w, bias, act):
    """Winograd F(2x2, 3x3) fp32 MFMA convolution (tsplat_conv3x3_wino_f32_fwd) against torch's
    conv2d in float64 on the CPU, with the launch's own workgroup shape choice and with each shape
    forced (TSPLAT_WINO_WG: 32 output channels / 4 waves, 64 / 8 waves, the 64-wide one padding
    co to 64; TSPLAT_WINO_KS: the 32-wide one with its chunks split over two 4-wave groups). The
    transforms reassociate the products (as MIOpen's Winograd solvers do), so the
    bound is 2e-5 of the output's max magnitude, like the direct kernel's."""
    from transplat_amd import kernels as K

    if wg != "auto":
        monkeypatch.setenv("TSPLAT_WINO_WG", wg[:2])
        monkeypatch.setenv("TSPLAT_WINO_KS", "2" if wg == "32x2" else "1")

    x = seeded((n, ci, h, w), 41)
    wt = seeded((co, ci, 3, 3), 42) * (1.0 / (9 * ci) ** 0.5)
    b = seeded((co,), 43) if bias else None
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double() if bias else None, padding=1)
    ref = {"none": ref, "relu": torch.relu(ref), "gelu": torch.nn.functional.gelu(ref)}[act].float()
    out = K.conv3x3_wino(x.to(device), wt.to(device), b.to(device) if bias else None, act).cpu()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err


def tf32_round(t: torch.Tensor) -> torch.Tensor:
    """fp32 -> TF32 (10 explicit mantissa bits, round to nearest even), as the reference's TF32
    convolutions / matmuls (src/main.py:15) see their operands."""
    i = t.float().contiguous().view(torch.int32)
    r = (i + 0xFFF + ((i >> 13) & 1)) & ~0x1FFF
    return r.view(torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("stage", ["auto", "0"])
@pytest.mark.parametrize("form", ["auto", "1", "2", "3", "4", "5", "6"])
@pytest.mark.parametrize("n,ci,co,h,w,bias,act", WINO_CASES + [(1, 24, 48, 10, 96, True, "relu"),
                                                               (2, 40, 64, 22, 136, False, "none"),
                                                               (3, 32, 40, 36, 64, True, "gelu"),
                                                               (2, 32, 32, 160, 160, True, "relu"),
                                                               # 64-wide form + its 32 x 32 tail launch
                                                               (2, 24, 84, 128, 128, True, "gelu")])
def test_conv3x3_wino_bf16x3_kernel(device, monkeypatch, stage, form, n, ci, co, h, w, bias, act):
    """Winograd F(2x2, 3x3) in split-bf16 precision (tsplat_conv3x3_wino_bf16x3_fwd: hi*hi + hi*lo +
    lo*hi on bf16 MFMA, fp32 accumulation) against torch's conv2d in float64, with the launch's own
    workgroup form and each form forced (TSPLAT_WINO3_FORM: 32 co x 32 tiles, the same with two
    k-groups, 32 x 64, 64 x 64, the persistent 32 x 32 form walking several tile blocks per workgroup
    across images -- staged maps only, else form 1 --, 64 x 32 with half the waves transforming), with
    the staged input (coalesced region loads through LDS, maps
    whose width is a multiple of 4: tile blocks 32 / 16 / 8 wide) and without it
    (TSPLAT_WINO3_STAGE=0). Bounds (written here): the same 2e-5 of max |y| as the exact-fp32
    kernel, and at most 1/8 of the error of the reference's own precision -- TF32 operands
    (float64 conv of TF32-rounded x and w, TF32's best case: exact accumulation)."""
    from transplat_amd import kernels as K

    if form != "auto":
        monkeypatch.setenv("TSPLAT_WINO3_FORM", form)
    if stage != "auto":
        monkeypatch.setenv("TSPLAT_WINO3_STAGE", stage)
    x = seeded((n, ci, h, w), 41)
    wt = seeded((co, ci, 3, 3), 42) * (1.0 / (9 * ci) ** 0.5)
    b = seeded((co,), 43) if bias else None
    fn = {"none": lambda t: t, "relu": torch.relu, "gelu": torch.nn.functional.gelu}[act]
    bd = b.double() if bias else None
    ref = fn(torch.nn.functional.conv2d(x.double(), wt.double(), bd, padding=1))
    ref_tf32 = fn(torch.nn.functional.conv2d(tf32_round(x).double(), tf32_round(wt).double(), bd, padding=1))
    args = (x.to(device), wt.to(device), b.to(device) if bias else None, act)
    out3 = K.conv3x3_wino(*args, precision="bf16x3").cpu().double()
    out32 = K.conv3x3_wino(*args, precision="fp32").cpu().double()
    scale = ref.abs().max().item()
    e3, e32, etf = ((o - ref).abs().max().item() / scale for o in (out3, out32, ref_tf32))
    print(f"wino bf16x3 form {form} {(n, ci, co, h, w)}: rel err {e3:.2e} (exact fp32 kernel {e32:.2e}, "
          f"TF32 operands {etf:.2e}; ratio to fp32 {e3 / max(e32, 1e-12):.1f}, to TF32 {e3 / etf:.3f})")
    assert e3 < 2e-5, e3
    assert e3 <= etf / 8, (e3, etf)


@pytest.mark.gpu
@pytest.mark.parametrize("stage", ["auto", "0"])
@pytest.mark.parametrize("n,c,h,w,skip", [(2, 128, 72, 72, True), (2, 128, 36, 36, False), (2, 128, 9, 9, True),
                                          (1, 64, 30, 52, True)])
def test_conv3x3_wino_bf16x3_relu_in_residual(device, monkeypatch, stage, n, c, h, w, skip):
    """The DPT ResidualConvUnit's fused form (tsplat_conv3x3_wino_bf16x3_ex_fwd): conv(relu(x)) +
    bias + x (+ the fusion block's skip) against float64, within 2e-5 of max |y|."""
    from transplat_amd import kernels as K

    if stage != "auto":
        monkeypatch.setenv("TSPLAT_WINO3_STAGE", stage)
    x = seeded((n, c, h, w), 91)
    wt = seeded((c, c, 3, 3), 92) * (1.0 / (9 * c) ** 0.5)
    b = seeded((c,), 93)
    sk = seeded((n, c, h, w), 94) if skip else None
    ref = torch.nn.functional.conv2d(torch.relu(x).double(), wt.double(), b.double(), padding=1) + x.double()
    if skip:
        ref = ref + sk.double()
    out = K.conv3x3_wino(x.to(device), wt.to(device), b.to(device), precision="bf16x3", residual=x.to(device),
                         residual2=sk.to(device) if skip else None, relu_in=True).cpu().double()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-5, err


@pytest.mark.gpu
@pytest.mark.parametrize("wgs", ["3", "7", "512"])
@pytest.mark.parametrize("chans", [(24, 16), (16, 16), (12, 8)])
def test_conv3x3_wino_bf16x3_persistent_walk(device, monkeypatch, wgs, chans):
    """The persistent form (TSPLAT_WINO3_FORM=5) with 3 / 7 / 512 workgroups per output block
    (TSPLAT_WINO3_PWG): each workgroup's flat (tile block, chunk) sequence crosses image and
    concatenation-source boundaries; ReLU-on-load and both residuals in the epilogue; against float64.
    Inputs of 40 channels (three 16-channel chunks) and of 32 / 20 (two chunks: the A fragments held
    in registers for the whole walk)."""
    from transplat_amd import kernels as K

    monkeypatch.setenv("TSPLAT_WINO3_FORM", "5")
    monkeypatch.setenv("TSPLAT_WINO3_PWG", wgs)
    ci = sum(chans)
    parts = [seeded((3, c, 40, 72), 120 + c + 7 * i) for i, c in enumerate(chans)]
    wt = seeded((48, ci, 3, 3), 131) * (1.0 / (9 * ci) ** 0.5)
    b = seeded((48,), 132)
    r1, r2 = seeded((3, 48, 40, 72), 133), seeded((3, 48, 40, 72), 134)
    x = torch.cat(parts, 1)
    ref = torch.nn.functional.conv2d(torch.relu(x).double(), wt.double(), b.double(), padding=1)
    ref = torch.nn.functional.gelu(ref) + r1.double() + r2.double()
    out = K.conv3x3_wino(parts[0].to(device), wt.to(device), b.to(device), "gelu", extra=(parts[1].to(device),),
                         precision="bf16x3", residual=r1.to(device), residual2=r2.to(device), relu_in=True)
    err = ((out.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-5, err


@pytest.mark.gpu
def test_conv3x3_wino_bf16x3_concat_and_production_size(device):
    """bf16x3 Winograd on the to_gaussians head's three sources at 256^2 (2 x 163 -> 168, the
    64 x 64 workgroup form) equals the kernel on the materialised concatenation bit for bit, and
    stays within 2e-5 of MIOpen's fp32 conv2d; the weight cache follows in-place updates."""
    from transplat_amd import kernels as K

    parts = [seeded((2, c, 256, 256), 60 + c).to(device) for c in (32, 3, 128)]
    wt = (seeded((168, 163, 3, 3), 63) * (1.0 / (9 * 163) ** 0.5)).to(device)
    b = seeded((168,), 64).to(device)
    y = K.conv3x3_wino(parts[0], wt, b, extra=tuple(parts[1:]), precision="bf16x3")
    cat = torch.cat(parts, 1)
    assert torch.equal(y, K.conv3x3_wino(cat, wt, b, precision="bf16x3"))
    ref = torch.nn.functional.conv2d(cat, wt, b, padding=1)
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 2e-5
    with torch.no_grad():
        wt.mul_(2.0)
    y2 = K.conv3x3_wino(cat, wt, None, precision="bf16x3")
    ref2 = torch.nn.functional.conv2d(cat, wt, None, padding=1)
    assert ((y2 - ref2).abs().max() / ref2.abs().max()).item() < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,bias,act", [(650, 768, 2304, True, "none"), (650, 768, 3072, True, "gelu"),
                                           (650, 3072, 768, True, "none"), (100, 256, 128, False, "none"),
                                           (8192, 256, 1024, False, "none"), (33, 64, 64, True, "gelu"),
                                           (20, 64, 128, True, "gelu")])
def test_linear_bf16x3_kernel(device, m, k, n, bias, act):
    """kernels.linear_bf16x3 (tsplat_split_bf16x3 + one hipBLASLt bf16 GEMM over K' = 3K, the
    correlation table's form) against float64 F.linear (+ exact GELU): within 2e-5 of max |y| and
    at most 1/8 of the TF32-operand error (tolerances written here); M not a multiple of a tile."""
    from transplat_amd import kernels as K

    x = seeded((m, k), 81)
    w = seeded((n, k), 82) / k ** 0.5
    b = seeded((n,), 83) if bias else None
    fn = torch.nn.functional.gelu if act == "gelu" else (lambda t: t)
    ref = fn(torch.nn.functional.linear(x.double(), w.double(), b.double() if bias else None))
    ref_tf = fn(torch.nn.functional.linear(tf32_round(x).double(), tf32_round(w).double(), b.double() if bias else None))
    out = K.linear_bf16x3(x.to(device), w.to(device), b.to(device) if bias else None, act=act).cpu().double()
    scale = ref.abs().max().item()
    e3, etf = (out - ref).abs().max().item() / scale, (ref_tf - ref).abs().max().item() / scale
    print(f"linear bf16x3 {(m, k, n)} {act}: rel err {e3:.2e}, TF32 operands {etf:.2e}")
    assert e3 < 2e-5 and e3 <= etf / 8, (e3, etf)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,bias,act", [(650, 768, 2304, True, "none"), (650, 768, 3072, True, "gelu"),
                                           (8192, 256, 1024, True, "none"), (8192, 128, 512, False, "none")])
def test_linear_xf32_library_path(device, monkeypatch, m, k, n, bias, act):
    """kernels.linear_xf32 (bf16x3 mode's library linears: hipBLASLt's emulated-xf32 GEMM under
    allow_tf32, then bias (+ exact GELU) in one pass) against float64: within 2e-5 of max |y| and at
    most 1/8 of the TF32-operand error -- the same bar as the split kernels; the shapes are the ones
    linear_xf32_ok admits (DINOv2 qkv / fc1, the transformer MLP input GEMMs). The route is off by
    default since round 6 (it raced in the graphed step, kernels._LINX); kept as the A/B form."""
    from transplat_amd import kernels as K

    monkeypatch.setattr(K, "_LINX", True)

    x = seeded((m, k), 91)
    w = seeded((n, k), 92) / k ** 0.5
    b = seeded((n,), 93) if bias else None
    fn = torch.nn.functional.gelu if act == "gelu" else (lambda t: t)
    ref = fn(torch.nn.functional.linear(x.double(), w.double(), b.double() if bias else None))
    ref_tf = fn(torch.nn.functional.linear(tf32_round(x).double(), tf32_round(w).double(), b.double() if bias else None))
    with K.dense_precision("bf16x3"):
        assert K.linear_xf32_ok(x.to(device), w.to(device))
        out = K.linear_xf32(x.to(device), w.to(device), b.to(device) if bias else None, act=act).cpu().double()
    assert not torch.backends.cuda.matmul.allow_tf32  # restored
    scale = ref.abs().max().item()
    e3, etf = (out - ref).abs().max().item() / scale, (ref_tf - ref).abs().max().item() / scale
    print(f"linear xf32 {(m, k, n)} {act}: rel err {e3:.2e}, TF32 operands {etf:.2e}")
    assert e3 < 2e-5 and e3 <= etf / 8, (e3, etf)


@pytest.mark.gpu
def test_conv3x3_wino_weight_cache_tracks_updates(device):
    """The transformed-filter cache is keyed on the live weight tensor and its version: an in-place
    update of the weight is picked up."""
    from transplat_amd import kernels as K

    x = seeded((1, 16, 8, 8), 44).to(device)
    wt = (seeded((16, 16, 3, 3), 45) * 0.1).to(device)
    y1 = K.conv3x3_wino(x, wt)
    with torch.no_grad():
        wt.mul_(2.0)
    y2 = K.conv3x3_wino(x, wt)
    torch.testing.assert_close(y2, 2.0 * y1, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_conv3x3_wino_reads_concat_in_place(device):
    """tsplat_conv3x3_wino_cat_f32_fwd on three sources (the to_gaussians head's cat of refine_out,
    images and the upsampled features: 32 + 3 + 128 channels) equals the kernel on the materialised
    concatenation bit for bit (same channel order, same arithmetic)."""
    from transplat_amd import kernels as K

    parts = [seeded((2, c, 20, 36), 50 + c).to(device) for c in (32, 3, 128)]
    wt = (seeded((84, 163, 3, 3), 53) * 0.03).to(device)
    b = seeded((84,), 54).to(device)
    y_cat = K.conv3x3_wino(parts[0], wt, b, "gelu", extra=tuple(parts[1:]))
    y_ref = K.conv3x3_wino(torch.cat(parts, 1), wt, b, "gelu")
    assert torch.equal(y_cat, y_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("co", [84, 96])
def test_conv3x3_wino_split_launch_at_production_size(device, co):
    """An odd number of 32-channel output blocks on a big grid (to_disparity's 168 -> 84 at 256^2)
    runs as a 64-channel launch for the even part plus a 32-channel launch for the last block
    (Args.cob_base); checked against MIOpen's fp32 conv2d."""
    from transplat_amd import kernels as K

    x = seeded((2, 168, 256, 256), 70).to(device)
    wt = (seeded((co, 168, 3, 3), 71) * (1.0 / (9 * 168) ** 0.5)).to(device)
    b = seeded((co,), 72).to(device)
    y = K.conv3x3_wino(x, wt, b, "gelu")
    ref = torch.nn.functional.gelu(torch.nn.functional.conv2d(x, wt, b, padding=1))
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 2e-5


@pytest.mark.gpu
def test_conv3x3_wino_wide_shape_at_production_size(device):
    """The launch picks the 64-output-channel workgroups for the to_gaussians head at 256^2
    (2 x 163 -> 168, three sources read in place); checked against MIOpen's fp32 conv2d on the
    materialised concatenation (the full-size float64 CPU reference would take minutes)."""
    from transplat_amd import kernels as K

    parts = [seeded((2, c, 256, 256), 60 + c).to(device) for c in (32, 3, 128)]
    wt = (seeded((168, 163, 3, 3), 63) * (1.0 / (9 * 163) ** 0.5)).to(device)
    b = seeded((168,), 64).to(device)
    y = K.conv3x3_wino(parts[0], wt, b, extra=tuple(parts[1:]))
    ref = torch.nn.functional.conv2d(torch.cat(parts, 1), wt, b, padding=1)
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 2e-5


@pytest.mark.gpu
def test_conv3x3_wino_ok_rejects_wide_input(device):
    """More input channels than the Winograd launch's plane table (kMaxCiPad = 1024 after padding to
    16) must route to MIOpen instead of reaching the kernel's EINVAL (advisor finding, round 2)."""
    from transplat_amd import kernels

    x = torch.randn(1, 1040, 20, 20, device=device)
    conv = torch.nn.Conv2d(1040, 32, 3, padding=1).to(device)
    assert not kernels.conv3x3_wino_ok(x, conv.weight, vs_miopen=True)
    with torch.no_grad():
        y = kernels.conv2d_forward(conv, x)
        ref = torch.nn.functional.conv2d(x, conv.weight, conv.bias, padding=1)
    torch.cuda.synchronize()
    assert (y - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


# ---------------------------------------------------------------- bf16 implicit-GEMM 3x3 / 1x1 (config C3)
# Reference: F.conv2d under bf16 autocast = conv of bf16-rounded sources / weights / bias with fp32
# accumulation, rounded to bf16. The check below is against the UNROUNDED float64 result of those
# bf16-rounded operands: the kernel's only differences are the fp32 summation order (<= 1e-5
# relative over <= 2304 exact products) and the final bf16 rounding (<= 2^-9 relative), so
# |y - ref| <= 2^-8 |ref| + 1e-4 max|ref| (tolerance written here, not a PSNR).
BF16_CASES = [
    # n, chans (sources), h, w (of the convolved map), cout, k, upsample, bias, act, src dtype
    (2, (32,), 64, 64, 32, 3, False, False, "none", "bf16"),        # U-Net 32-ch level (CT = 1, TW = 64)
    (2, (128,), 32, 32, 128, 3, False, False, "none", "bf16"),      # 128-ch level (CT = 2, TW = 32)
    (2, (128, 128), 16, 16, 128, 3, False, False, "none", "bf16"),  # output block on cat([h, skip]) (TW = 16)
    (2, (64, 32), 16, 16, 32, 3, False, True, "silu", "f32"),       # fp32 sources rounded on load, 2 sources
    (1, (96,), 24, 24, 96, 3, False, True, "gelu", "f32"),          # co % 64 != 0, W = 24 (partial 16-col tiles)
    (1, (64,), 128, 128, 64, 3, False, True, "relu", "bf16"),       # depth-predictor head shape (scaled down)
    (3, (8,), 9, 8, 40, 3, False, True, "none", "bf16"),            # TW = 8, H not a multiple of TH, tiny cin
    (1, (40, 16, 8), 20, 72, 33, 3, False, True, "gelu", "f32"),    # 3 sources, ci = 64 + pad, W = 72 (2 x-tiles)
    (2, (256,), 32, 32, 128, 1, False, True, "none", "bf16"),       # ResBlock 1x1 skip
    (2, (128, 64), 16, 16, 96, 1, False, True, "none", "f32"),      # 1x1 on a concat, co % 64 != 0
    (2, (128,), 32, 32, 128, 3, True, True, "none", "bf16"),        # Upsample: nearest 2x (16^2 -> 32^2) + 3x3
    (1, (32,), 64, 16, 32, 3, True, True, "none", "f32"),           # upsample, fp32 source, TW = 16
    (2, (32, 3, 128), 64, 64, 96, 3, False, True, "gelu", "mix"),   # to_gaussians head: ragged + mixed dtypes
    (1, (3, 1, 20, 1, 1), 32, 32, 40, 3, False, False, "none", "mix"),  # 5 ragged sources: rejected (> 4)
    (2, (5, 12), 16, 16, 32, 3, True, True, "silu", "mix"),         # ragged + upsample
    (1, (32, 3, 128), 64, 64, 168, 3, False, True, "gelu", "mix"),  # register-blocked form (ci co >= 96^2), co % 64 != 0
    (2, (128,), 40, 32, 128, 3, False, False, "none", "bf16"),      # register-blocked form, TW = 32, H % TH != 0
]


def _bf16_ref(srcs, w, b, act, up):
    x = torch.cat([s.double().bfloat16().double() if s.dtype == torch.float32 else s.double() for s in srcs], 1)
    if up:
        x = torch.nn.functional.interpolate(x, scale_factor=2, mode="nearest")
    wr = w.bfloat16().double()
    br = b.bfloat16().double() if b is not None else None
    y = torch.nn.functional.conv2d(x, wr, br, padding=w.shape[-1] // 2)
    return {"none": y, "relu": torch.relu(y), "silu": torch.nn.functional.silu(y),
            "gelu": torch.nn.functional.gelu(y)}[act]


@pytest.mark.parametrize("k", [3, 1])
def test_conv_bf16_weight_packing_layout(k):
    """Host-side packing (kernels.conv_bf16_pack_weight) against the A-operand map the kernel
    reads: lane c + 32 h of block b, chunk j, tap holds w[32 b + c][16 j + 8 h + e][tap], zero pad."""
    from transplat_amd import kernels as K
    import transplat_amd._lib as L

    co, ci, taps = 40, 24, k * k
    w = seeded((co, ci, k, k), 5)
    p = K.conv_bf16_pack_weight(w).view(2, 2, taps, 64, 8)
    wb = w.bfloat16().reshape(co, ci, taps)
    for b, j, tap, lane, e in [(0, 0, 0, 0, 0), (0, 1, 4, 37, 3), (1, 0, 8, 7, 7), (1, 1, 2, 63, 5), (0, 0, 5, 40, 6)]:
        tap = tap % taps
        c, h = lane % 32, lane // 32
        o, i = 32 * b + c, 16 * j + 8 * h + e
        want = wb[o, i, tap] if (o < co and i < ci) else torch.zeros((), dtype=torch.bfloat16)
        assert p[b, j, tap, lane, e] == want, (b, j, tap, lane, e)
    # byte count = the C-ABI's tsplat_conv2d_bf16_weight_bytes formula
    assert K.conv_bf16_pack_weight(w).numel() * 2 == 2 * 2 * taps * 64 * 16
    assert "tsplat_conv2d_bf16_weight_bytes" in L.SIGNATURES


@pytest.mark.gpu
@pytest.mark.parametrize("n,chans,h,w,cout,k,up,has_bias,act,sdt", BF16_CASES)
def test_conv_bf16_kernel(device, n, chans, h, w, cout, k, up, has_bias, act, sdt):
    from transplat_amd import kernels as K

    hs, ws = (h // 2, w // 2) if up else (h, w)
    dts = [torch.float32 if (sdt == "f32" or (sdt == "mix" and i % 2)) else torch.bfloat16 for i in range(len(chans))]
    srcs = [seeded((n, c, hs, ws), 300 + i).to(dts[i]) for i, c in enumerate(chans)]
    wt = seeded((cout, sum(chans), k, k), 310) * 0.1
    b = seeded((cout,), 311) if has_bias else None
    ref = _bf16_ref(srcs, wt, b, act, up)
    dsrc = [s.to(device) for s in srcs]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        if len(chans) > 4:
            assert not K.conv_bf16_ok(dsrc[0], wt, extra=tuple(dsrc[1:]), upsample=up)
            return
        assert K.conv_bf16_ok(dsrc[0], wt, extra=tuple(dsrc[1:]), upsample=up)
        y = K.conv_bf16(dsrc[0], wt.to(device), b.to(device) if b is not None else None, act, extra=tuple(dsrc[1:]),
                        upsample=up)
    assert y.dtype == torch.bfloat16 and tuple(y.shape) == (n, cout, h, w)
    err = (y.double().cpu() - ref).abs()
    bound = 2.0 ** -8 * ref.abs() + 1e-4 * ref.abs().max()
    assert bool((err <= bound).all()), f"max excess {(err - bound).max():.3e}"


@pytest.mark.gpu
def test_conv_bf16_module_routes(device):
    """Under bf16 autocast the U-Net conv helper (plain, 1x1, upsample) and the installed Conv2d
    dispatch take the bf16 kernel (bf16 output, no MIOpen call), matching F.conv2d under autocast to
    bf16 rounding."""
    from transplat_amd import kernels as K
    from transplat_amd.model.encoder.matching import ldm_unet as U

    conv = torch.nn.Conv2d(64, 64, 3, 1, 1).to(device)
    conv1 = torch.nn.Conv2d(64, 32, 1).to(device)
    conv1d = torch.nn.Conv1d(64, 96, 1).to(device)
    t = seeded((2, 64, 256), 321).to(device)
    x = seeded((2, 64, 32, 32), 320).to(device)
    F = torch.nn.functional
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        cases = [(U.conv(conv, x), F.conv2d(x, conv.weight, conv.bias, padding=1)),
                 (K.conv2d_forward(conv, x), F.conv2d(x, conv.weight, conv.bias, padding=1)),
                 (U.conv(conv1, x), F.conv2d(x, conv1.weight, conv1.bias)),
                 (U.conv(conv1d, t), F.conv1d(t, conv1d.weight, conv1d.bias)),
                 (U.conv(conv, x, upsample=True),
                  F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), conv.weight, conv.bias, padding=1))]
    for y, ref in cases:
        assert y.dtype == torch.bfloat16 and y.shape == ref.shape
        assert (y.float() - ref.float()).abs().max() <= 2 * 2.0 ** -8 * ref.float().abs().max()


@pytest.mark.gpu
def test_conv_bf16_rejects_unsupported(device):
    from transplat_amd import kernels as K

    w = torch.zeros(32, 32, 3, 3, device=device)
    x = torch.zeros(1, 32, 16, 16, device=device)
    assert not K.conv_bf16_ok(x, w)  # autocast off
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert K.conv_bf16_ok(x, w)
        assert not K.conv_bf16_ok(torch.zeros(1, 32, 16, 12, device=device), w)   # width % 8
        assert not K.conv_bf16_ok(x, w, stride=2)
        assert not K.conv_bf16_ok(x, torch.zeros(32, 32, 5, 5, device=device))
        assert K.conv_bf16_ok(torch.zeros(1, 36, 16, 16, device=device), torch.zeros(32, 36, 3, 3, device=device))
        assert not K.conv_bf16_ok(torch.zeros(1, 36, 16, 16, device=device), torch.zeros(32, 35, 3, 3, device=device))
        assert not K.conv_bf16_ok(x.contiguous(memory_format=torch.channels_last), w)
        assert not K.conv_bf16_ok(torch.zeros(1, 32, 16, 6, device=device), w, upsample=True)  # 12 % 8


X3_CASES = CASES + [
    (1, 3, 5, 9, 13, 40, 3, 1, False, True),          # odd channel counts (the split kernel's 16-groups)
    (2, 768, 0, 9, 9, 128, 3, 1, False, True),        # long reduction -> zsplit
    (2, 256, 0, 64, 64, 128, 1, 1, False, True),
    (2, 768, 0, 18, 18, 768, 3, 2, False, True),      # the DPT's stride-2 768-channel level
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,c1,c2,h,w,cout,k,stride,up,has_bias", X3_CASES)
def test_conv2d_direct_bf16x3_kernel(device, monkeypatch, n, c1, c2, h, w, cout, k, stride, up, has_bias):
    """tsplat_conv2d_bf16x3_fwd (the direct convolution in the bf16x3 dense mode) against float64:
    within 2e-5 of max |y| AND at most 1/8 of the error of TF32-rounded operands (the reference's
    own arithmetic, src/main.py:15) on the same inputs; bit-identical over repeated launches. Every
    case forced onto the split kernel (the dispatch keeps the small 3x3s exact fp32)."""
    from transplat_amd import kernels as K

    monkeypatch.setattr(K, "conv_x3_wins", lambda *a: True)

    F = torch.nn.functional
    x1 = seeded((n, c1, h, w), 11)
    x2 = seeded((n, c2, h, w), 12) if c2 else None
    wt = seeded((cout, c1 + c2, k, k), 13) * (1.0 / (c1 + c2) ** 0.5)
    b = seeded((cout,), 14) if has_bias else None

    def ref_of(a1, a2, ww):
        x = torch.cat([a1, a2], 1) if a2 is not None else a1
        if up:
            x = F.interpolate(x, scale_factor=2, mode="nearest")
        return F.conv2d(x.double(), ww.double(), b.double() if b is not None else None, stride, padding=k // 2)

    ref = ref_of(x1, x2, wt)
    ref_tf = ref_of(tf32_round(x1), tf32_round(x2) if x2 is not None else None, tf32_round(wt))
    args = (x1.to(device), wt.to(device), b.to(device) if b is not None else None, stride)
    with K.dense_precision("bf16x3"):
        outs = [K.conv2d_direct(*args, x2=x2.to(device) if x2 is not None else None, upsample=up).cpu()
                for _ in range(2)]
    scale = ref.abs().max().item()
    err = (outs[0].double() - ref).abs().max().item() / scale
    etf = (ref_tf - ref).abs().max().item() / scale
    print(f"direct bf16x3 {(n, c1, c2, h, w, cout, k, stride, up)}: rel err {err:.2e} (TF32 operands {etf:.2e})")
    assert err < 2e-5 and err <= etf / 8, (err, etf)
    assert torch.equal(outs[0], outs[1])


FEW_CASES = [
    # n, source channels, co, h, w, act, relu_in, residuals
    (2, (32,), 32, 256, 256, "none", False, 0),      # refine U-Net 256^2 ResBlock conv
    (2, (64,), 32, 256, 256, "none", False, 0),      # its output block on cat([h, skip]) (one source here)
    (2, (32, 32), 32, 256, 256, "none", False, 0),   # ... read as two sources in place
    (2, (3, 1, 32, 1, 1), 32, 256, 256, "none", False, 0),  # the refine input cat (38 channels, 5 sources)
    (2, (32,), 64, 256, 256, "gelu", False, 0),      # to_disparity conv 1 (+ GELU)
    (2, (64,), 2, 256, 256, "none", False, 0),       # to_disparity conv 2 (2 of 32 columns used)
    (2, (32,), 32, 128, 128, "none", False, 0),      # 128^2 level (4-row blocks)
    (2, (64,), 64, 128, 128, "relu", True, 2),       # relu-on-load, both residuals
    (1, (40,), 48, 36, 252, "none", False, 1),       # ragged: h % 8, w % 64 != 0, co % 32 != 0
    (3, (96, 32), 16, 20, 68, "gelu", False, 0),     # 128 input channels (4 passes), tiny map (2-row form)
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,chans,co,h,w,act,relu_in,nres", FEW_CASES)
def test_conv3x3_few_kernel(device, n, chans, co, h, w, act, relu_in, nres):
    """tsplat_conv3x3_few_bf16x3_fwd (direct split-bf16 3x3 for few-channel full-resolution maps,
    csrc/convfew.hip) against torch's conv2d in float64: the same bounds as the bf16x3 Winograd kernel
    (2e-5 of max |y|, and <= 1/8 of the TF32-operand error). The launch is checked to take the direct
    kernel (tsplat_conv3x3_few_form)."""
    from transplat_amd import _lib
    from transplat_amd import kernels as K

    ci = sum(chans)
    assert int(_lib.load().tsplat_conv3x3_few_form(n, ci, h, w, co)) != 0
    parts = [seeded((n, c, h, w), 150 + 3 * i + c) for i, c in enumerate(chans)]
    x = torch.cat(parts, 1)
    wt = seeded((co, ci, 3, 3), 161) * (1.0 / (9 * ci) ** 0.5)
    b = seeded((co,), 162)
    res = [seeded((n, co, h, w), 163 + i) for i in range(nres)]
    fn = {"none": lambda t: t, "relu": torch.relu, "gelu": torch.nn.functional.gelu}[act]
    xin = torch.relu(x) if relu_in else x
    ref = fn(torch.nn.functional.conv2d(xin.double(), wt.double(), b.double(), padding=1))
    ref_tf32 = fn(torch.nn.functional.conv2d(tf32_round(xin).double(), tf32_round(wt).double(), b.double(),
                                             padding=1))
    for r in res:
        ref, ref_tf32 = ref + r.double(), ref_tf32 + r.double()
    lib = _lib.load()
    import ctypes

    srcs = [p.to(device).contiguous() for p in parts]
    y = torch.empty((n, co, h, w), device=device)
    ptrs = (ctypes.c_void_p * len(srcs))(*[t.data_ptr() for t in srcs])
    cs = (ctypes.c_int32 * len(srcs))(*chans)
    rd = [r.to(device) for r in res] + [None, None]
    rc = lib.tsplat_conv3x3_few_bf16x3_fwd(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(cs, ctypes.c_void_p),
                                           len(srcs), K.conv_pack_weight_x3(wt.to(device)).data_ptr(),
                                           b.to(device).data_ptr(), _lib.ptr(rd[0]), _lib.ptr(rd[1]), y.data_ptr(),
                                           n, h, w, co, {"none": 0, "relu": 1, "gelu": 2}[act], int(relu_in),
                                           _lib.stream_ptr(device))
    assert rc == 0
    out = y.cpu().double()
    scale = ref.abs().max().item()
    e3, etf = ((o - ref).abs().max().item() / scale for o in (out, ref_tf32))
    print(f"few-channel conv {(n, chans, co, h, w, act, relu_in, nres)}: rel err {e3:.2e} (TF32 operands {etf:.2e})")
    assert e3 < 2e-5, e3
    assert e3 <= etf / 8, (e3, etf)


@pytest.mark.gpu
def test_conv3x3_few_route_matches_kernel(device):
    """kernels.conv3x3_wino in the bf16x3 mode takes the direct few-channel kernel for a refine-U-Net
    shape (same bits as the C-ABI call above would give), and the Winograd one with TSPLAT_CONV_FEW off;
    both within the bf16x3 bound of float64."""
    from transplat_amd import kernels as K

    x = seeded((2, 32, 256, 256), 171).to(device)
    wt = (seeded((32, 32, 3, 3), 172) / 17.0).to(device)
    b = seeded((32,), 173).to(device)
    with K.dense_precision("bf16x3"):
        assert K._few_ok([x], 2, 256, 256, 32)
        y_few = K.conv3x3_wino(x, wt, b)
        K._FEW = False
        try:
            y_w = K.conv3x3_wino(x, wt, b)
        finally:
            K._FEW = True
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), padding=1)
    s = ref.abs().max().item()
    assert (y_few.double() - ref).abs().max().item() / s < 2e-5
    assert (y_w.double() - ref).abs().max().item() / s < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,bias,act,ksplit", [
    (650, 768, 2304, True, "none", 1), (650, 768, 3072, True, "gelu", 1), (650, 3072, 768, True, "none", 4),
    (650, 768, 768, True, "none", 0), (650, 3072, 768, False, "none", 48), (33, 72, 100, True, "gelu", 1),
    (1, 4, 4, False, "none", 1), (8192, 256, 1024, True, "none", 1), (130, 200, 260, True, "none", 2)])
def test_gemm_x3_kernel(device, m, k, n, bias, act, ksplit):
    """tsplat_gemm_x3_fwd (the bf16x3 mode's DINOv2 linears) against float64: the sum of its split-K
    slabs within 2e-5 of max |y| and at most 1/8 of the TF32-operand error (the bar of the other
    split kernels); ragged m / n / k (tile, chunk and split edges), every split a partial product
    with the bias only in slab 0, the exact-GELU epilogue; two launches bit-identical."""
    from transplat_amd import kernels as K

    x = seeded((m, k), 191)
    w = seeded((n, k), 192) / k ** 0.5
    b = seeded((n,), 193) if bias else None
    fn = torch.nn.functional.gelu if act == "gelu" else (lambda t: t)
    ref = fn(torch.nn.functional.linear(x.double(), w.double(), b.double() if bias else None))
    ref_tf = fn(torch.nn.functional.linear(tf32_round(x).double(), tf32_round(w).double(), b.double() if bias else None))
    xd, wd = x.to(device), w.to(device)
    with K.dense_precision("bf16x3"):
        assert K.gemm_x3_ok(xd, wd)
        y = K.gemm_x3(xd, wd, b.to(device) if bias else None, act=act, ksplit=ksplit)
        y2 = K.gemm_x3(xd, wd, b.to(device) if bias else None, act=act, ksplit=ksplit)
    s = ksplit if ksplit else K.gemm_ksplit(m, n, k)
    assert y.shape == ((m, n) if s == 1 else (s, m, n))
    assert torch.equal(y, y2)
    out = (y.double().sum(0) if s > 1 else y.double()).cpu()
    scale = ref.abs().max().item()
    e3, etf = (out - ref).abs().max().item() / scale, (ref_tf - ref).abs().max().item() / scale
    print(f"gemm x3 {(m, k, n)} {act} ksplit {s}: rel err {e3:.2e}, TF32 operands {etf:.2e}")
    assert e3 < 2e-5 and e3 <= etf / 8, (e3, etf)


@pytest.mark.gpu
def test_residual_ln_slabs(device):
    """tsplat_residual_ln_slabs_fwd == tsplat_residual_ln_fwd on the slabs' sum (summed in slab order,
    bit for bit against the same order in fp32)."""
    from transplat_amd import kernels as K

    x = seeded((2, 325, 768), 201).to(device)
    y = seeded((4, 2, 325, 768), 202).to(device)
    ls = seeded((768,), 203).to(device)
    norm = torch.nn.LayerNorm(768, eps=1e-6).to(device)
    with torch.no_grad():
        norm.weight.copy_(seeded((768,), 204))
        norm.bias.copy_(seeded((768,), 205))
    xs, ns = K.residual_ln(x, y, ls, norm)
    ysum = ((y[0] + y[1]) + y[2]) + y[3]
    xr, nr = K.residual_ln(x, ysum, ls, norm)
    assert torch.equal(xs, xr) and torch.equal(ns, nr)


@pytest.mark.gpu
def test_gemm_x3_split_output_feeds_mha(device):
    """gemm_x3(act="split") writes x W^T + bias as hi / lo bf16 images equal (bit for bit) to splitting
    the fp32 output; tsplat_mha_x3_presplit_fwd on them == tsplat_mha_x3_fwd on the fp32 qkv (DINOv2's
    qkv -> attention hand-off, 2 x 325 tokens, 12 heads)."""
    from transplat_amd import kernels as K

    x = seeded((2, 325, 768), 211).to(device)
    w = (seeded((2304, 768), 212) / 768 ** 0.5).to(device)
    b = seeded((2304,), 213).to(device)
    with K.dense_precision("bf16x3"):
        y = K.gemm_x3(x, w, b)
        sp = K.gemm_x3(x, w, b, act="split")
        hi = y.to(torch.bfloat16)
        lo = (y - hi.float()).to(torch.bfloat16)
        assert torch.equal(sp[0], hi) and torch.equal(sp[1], lo)
        o_ref = K.mha(y, 12, 0.125)
        o = K.mha_presplit(sp, 12, 0.125)
    assert torch.equal(o, o_ref)
