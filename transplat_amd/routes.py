"""What actually ran: a route census of one step, for the bench line's workload string.

`record()` observes one eager step from two sides:
- every C-ABI call (`_lib.check` notes the entry point and, where a flag picks the arithmetic, the
  precision the call site passed), and
- every ATen op that reaches a vendor library (a TorchDispatchMode: `aten.convolution` -> MIOpen,
  `mm` / `addmm` / `bmm` / `baddbmm` -> hipBLASLt), with its operand dtype and the matmul mode
  in force (allow_tf32 = hipBLASLt's emulated xf32; bf16 operands in the bf16x3 dense mode = the
  split-bf16 K = 3k GEMMs; bf16 under autocast = plain bf16).

`Routes.label()` turns the census into the precision statement (what runs in which arithmetic, and
what is left on a library), so the bench's `config.workload` is derived, not hand-written (VERDICT r5
weak #4: the hand-written string said "DPT-head 3x3s on MIOpen" after they had moved to Winograd).
"""
from __future__ import annotations

from collections import Counter
from contextlib import contextmanager

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from . import _lib

# C-ABI entry point -> (category, arithmetic); None arithmetic = given by the call site (`route=`)
_HIP = {
    "tsplat_win_attn_x3_partials_fwd": ("window attention", "bf16x3 (split-bf16 products, fp32 softmax)"),
    "tsplat_win_attn_x3_fwd": ("window attention", "bf16x3 (split-bf16 products, fp32 softmax)"),
    "tsplat_win_attn_bf16_shift_fwd": ("window attention", "bf16 MFMA, fp32 softmax"),
    "tsplat_win_attn_bf16_fwd": ("window attention", "bf16 MFMA, fp32 softmax"),
    "tsplat_win_attn_partials_fwd": ("window attention", "exact fp32"),
    "tsplat_win_attn_fwd": ("window attention", "exact fp32"),
    "tsplat_conv3x3_wino_bf16x3_fwd": ("3x3 convs (HIP Winograd)", "bf16x3"),
    "tsplat_conv3x3_wino_bf16x3_ex_fwd": ("3x3 convs (HIP Winograd)", "bf16x3"),
    "tsplat_conv3x3_wino_bf16x3_cat_fwd": ("3x3 convs (HIP Winograd)", "bf16x3"),
    "tsplat_conv3x3_wino_f32_fwd": ("3x3 convs (HIP Winograd)", "exact fp32"),
    "tsplat_conv3x3_wino_cat_f32_fwd": ("3x3 convs (HIP Winograd)", "exact fp32"),
    "tsplat_conv3x3_few_bf16x3_fwd": ("direct convs (HIP)", "bf16x3"),
    "tsplat_conv2d_bf16x3_fwd": ("direct convs (HIP)", "bf16x3"),
    "tsplat_conv2d_f32_fwd": ("direct convs (HIP)", "exact fp32"),
    "tsplat_conv2d_f32_zsplit_fwd": ("direct convs (HIP)", "exact fp32"),
    "tsplat_conv2d_f32_nhwc_fwd": ("direct convs (HIP)", "exact fp32"),
    "tsplat_conv2d_bf16_fwd": ("direct convs (HIP)", "bf16"),
    "tsplat_linear_f32_fwd": ("transformer linears (HIP)", None),
    "tsplat_linear_f32_split_x3_fwd": ("transformer linears (HIP)", None),
    "tsplat_linear_f32_attn_merge_fwd": ("transformer linears (HIP)", None),
    "tsplat_gemm_x3_fwd": ("GEMMs (HIP)", "bf16x3"),
    "tsplat_mha_x3_fwd": ("DINOv2 attention (HIP)", "bf16x3"),
    "tsplat_mha_x3_presplit_fwd": ("DINOv2 attention (HIP)", "bf16x3"),
    "tsplat_mha_f32_fwd": ("DINOv2 attention (HIP)", "exact fp32"),
    "tsplat_mha_bias_f32_fwd": ("DINOv2 attention (HIP)", "exact fp32"),
    "tsplat_qkv_attention_cf_fwd": ("U-Net attention (HIP)", "exact fp32"),
    "tsplat_uv_coarse_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_uv_cross_table_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_uv_cross_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_msda_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_msda_raw_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_ms_deform_attn_fwd": ("correlation (HIP)", "fp32"),
    "tsplat_group_norm_fwd": ("norms (HIP)", "fp32"),
    "tsplat_group_norm_cat_res_fwd": ("norms (HIP)", "fp32"),
    "tsplat_group_norm_bf16_fwd": ("norms (HIP)", "bf16 I/O, fp32 statistics"),
    "tsplat_layer_norm128_fwd": ("norms (HIP)", None),
    "tsplat_residual_ln_fwd": ("norms (HIP)", "fp32"),
    "tsplat_residual_ln_slabs_fwd": ("norms (HIP)", "fp32"),
    "tsplat_residual_ln_bf16_fwd": ("norms (HIP)", "bf16 I/O, fp32 statistics"),
    "tsplat_gaussian_adapter_fwd": ("gaussian adapter (HIP)", "fp32"),
    "tsplat_sh_rotation_fwd": ("gaussian adapter (HIP)", "fp32"),
    "tsplat_raster_fwd": ("rasterizer (HIP)", "fp32"),
}
_ORDER = ("window attention", "transformer linears (HIP)", "GEMMs (HIP)", "3x3 convs (HIP Winograd)", "direct convs (HIP)",
          "DINOv2 attention (HIP)", "U-Net attention (HIP)", "library GEMMs (hipBLASLt)", "library convs (MIOpen)",
          "correlation (HIP)", "norms (HIP)", "gaussian adapter (HIP)", "rasterizer (HIP)")
_GEMMS = {"mm", "addmm", "bmm", "baddbmm", "addbmm", "_scaled_mm"}
_CONVS = {"convolution", "_convolution", "cudnn_convolution", "miopen_convolution", "convolution_overrideable",
          "conv2d", "conv_transpose2d", "miopen_convolution_transpose"}


class Routes:
    def __init__(self):
        self.calls: Counter = Counter()  # (category, arithmetic) -> launches
        self.library: list = []  # (op, dtype, shapes) of every library call

    def note(self, what: str, route: str | None = None) -> None:
        cat = _HIP.get(what)
        if cat is None:
            return
        self.calls[(cat[0], route or cat[1] or "?")] += 1

    def lib(self, op: str, arith: str, shapes) -> None:
        cat = "library GEMMs (hipBLASLt)" if op in _GEMMS else "library convs (MIOpen)"
        self.calls[(cat, arith)] += 1
        self.library.append((op, arith, shapes))

    def by_category(self) -> dict:
        out: dict = {}
        for (cat, arith), n in self.calls.items():
            out.setdefault(cat, Counter())[arith] += n
        return out

    def label(self) -> str:
        cats = self.by_category()
        parts = []
        for cat in _ORDER:
            if cat == "library convs (MIOpen)" and cat not in cats:
                parts.append("library convs (MIOpen): none")
                continue
            if cat not in cats:
                continue
            items = ", ".join(f"{a} x{n}" for a, n in sorted(cats[cat].items(), key=lambda kv: -kv[1]))
            parts.append(f"{cat}: {items}")
        return "; ".join(parts)


class _LibraryOps(TorchDispatchMode):
    def __init__(self, routes: Routes):
        super().__init__()
        self.routes = routes

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func.overloadpacket.__name__
        if name in _GEMMS or name in _CONVS:
            ts = [a for a in args if torch.is_tensor(a)]
            if ts and ts[0].is_cuda:
                dt = ts[-1].dtype if name in _GEMMS else ts[0].dtype
                if name in _GEMMS and dt == torch.float32:
                    arith = "xf32 (emulated, bf16 MFMA)" if torch.backends.cuda.matmul.allow_tf32 else "exact fp32"
                elif name in _GEMMS and dt == torch.bfloat16:
                    from . import kernels

                    arith = ("bf16x3 (split-bf16 K = 3k)" if kernels.split_mode()
                             and not torch.is_autocast_enabled("cuda") else "bf16")
                else:
                    arith = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}.get(dt, str(dt))
                shapes = [tuple(t.shape) for t in ts]
                if name in _CONVS and len(args) >= 7:  # + (stride, padding, transposed)
                    shapes.append((tuple(args[3]), tuple(args[4]), bool(args[6])))
                self.routes.lib(name, arith, shapes)
        return func(*args, **kwargs)


@contextmanager
def record():
    """Census of everything launched inside the block (eager only: no hipGraph capture)."""
    routes = Routes()
    prev = _lib.ROUTE_HOOK
    _lib.ROUTE_HOOK = routes.note
    try:
        with _LibraryOps(routes):
            yield routes
    finally:
        _lib.ROUTE_HOOK = prev
