"""ctypes binding of the C-ABI in include/transplat_hip.h.

The product path has exactly one implementation: the gfx950 HIP library built in-tree
(`transplat_amd/libtransplat_hip.so`). There is no CPU or PyTorch fallback; if the library is
missing or a tensor is not on a HIP device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

# TSPLAT_LIB (benchmarking only) points at an alternative build of the same library
_LIB_PATH = Path(os.environ.get("TSPLAT_LIB") or Path(__file__).resolve().parent / "libtransplat_hip.so")
_lib = None


class RasterDesc(ctypes.Structure):
    _fields_ = [
        ("num_gaussians", ctypes.c_int32),
        ("num_views", ctypes.c_int32),
        ("views_per_scene", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("sh_coeffs", ctypes.c_int32),
        ("sh_degree", ctypes.c_int32),
        ("capacity", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32

# name -> (restype, argtypes); must match include/transplat_hip.h exactly
SIGNATURES = {
    "tsplat_version": (ctypes.c_int, []),
    "tsplat_set_debug": (ctypes.c_int, [_I32]),
    "tsplat_timestamp": (ctypes.c_int, [_P, _I32, _P]),
    "tsplat_prof_enable": (ctypes.c_int, [_I32]),
    "tsplat_prof_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I32)]),
    "tsplat_raster_workspace_bytes": (ctypes.c_size_t, [_I32, _I32, _I32, _I32, _I32]),
    "tsplat_raster_num_rendered_offset": (ctypes.c_size_t, [_I32, _I32, _I32, _I32]),
    "tsplat_raster_fwd": (
        ctypes.c_int,
        [ctypes.POINTER(RasterDesc)] + [_P] * 15,
    ),
    "tsplat_uv_coarse_fwd": (ctypes.c_int, [_P] * 4 + [_I32] * 5 + [_P]),
    "tsplat_uv_cross_fwd": (ctypes.c_int, [_P] * 7 + [_I32] * 6 + [_P]),
    "tsplat_uv_cross_table_fwd": (ctypes.c_int, [_P] * 6 + [_I32] * 6 + [_P]),
    "tsplat_msda_fwd": (ctypes.c_int, [_P] * 4 + [_I32] * 6 + [_P]),
    "tsplat_msda_raw_fwd": (ctypes.c_int, [_P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_ms_deform_attn_fwd": (ctypes.c_int, [_P] * 6 + [_I32] * 8 + [_P]),
    "tsplat_win_attn_workspace_bytes": (ctypes.c_size_t, [_I32] * 5),
    "tsplat_win_attn_fwd": (ctypes.c_int, [_P] * 5 + [_I32] * 7 + [_P]),
    "tsplat_win_attn_bf16_workspace_bytes": (ctypes.c_size_t, [_I32] * 5),
    "tsplat_win_attn_bf16_fwd": (ctypes.c_int, [_P] * 5 + [_I32] * 7 + [_P]),
    "tsplat_win_attn_bf16_shift_fwd": (ctypes.c_int, [_P] * 5 + [_I32] * 8 + [_P]),
    "tsplat_group_norm_workspace_bytes": (ctypes.c_size_t, [_I32, _I32, ctypes.c_int64, _I32]),
    "tsplat_group_norm_fwd": (ctypes.c_int, [_P] * 7 + [_I32, _I32, ctypes.c_int64, _I32, ctypes.c_float, _I32, _P]),
    "tsplat_group_norm_cat_res_fwd": (ctypes.c_int, [_P] * 6 + [_I32, _P, _P, _I32, _I32, ctypes.c_int64, _I32,
                                                                ctypes.c_float, _I32, _P]),
    "tsplat_layer_norm128_fwd": (ctypes.c_int, [_P, _I32, _P, _P, _P, ctypes.c_float, _P, _I32, _I32, _P]),
    "tsplat_group_norm_bf16_fwd": (ctypes.c_int, [_P] * 7 + [_I32, _I32, ctypes.c_int64, _I32, ctypes.c_float, _I32,
                                                            _P]),
    "tsplat_sh_rotation_fwd": (ctypes.c_int, [_P] * 3 + [_I32] * 2 + [_P]),
    "tsplat_gaussian_adapter_fwd": (ctypes.c_int, [_P] * 9 + [_I32] * 6 + [ctypes.c_float] * 3 + [_I32, _I32, _P]),
    "tsplat_win_attn_split": (_I32, [_I32] * 5),
    "tsplat_depth_softmax_fwd": (ctypes.c_int, [_P] * 4 + [_I32] * 3 + [_P]),
    "tsplat_depth_tail_fwd": (ctypes.c_int, [_P] * 6 + [_I32] * 3 + [_P]),
    "tsplat_raster_cameras": (ctypes.c_int, [_P] * 5 + [_I32] * 3 + [_P] * 7),
    "tsplat_small_inverse": (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    "tsplat_mha_f32_fwd": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, ctypes.c_float, _P]),
    "tsplat_mha_bias_f32_fwd": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_float, _P]),
    "tsplat_mha_x3_workspace_bytes": (ctypes.c_size_t, [_I32] * 4),
    "tsplat_mha_x3_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_float, _P]),
    "tsplat_mha_x3_presplit_fwd": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_float, _P]),
    "tsplat_qkv_attention_cf_fwd": (ctypes.c_int, [_P, _P] + [_I32] * 5 + [ctypes.c_float, _P]),
    "tsplat_conv2d_f32_fwd": (ctypes.c_int, [_P, _I32, _P, _I32, _P, _P, _P] + [_I32] * 8 + [_P]),
    "tsplat_conv2d_f32_zsplit_fwd": (ctypes.c_int, [_P, _I32, _P, _I32, _P, _P, _P] + [_I32] * 9 + [_P, _P, _P]),
    "tsplat_conv2d_bf16x3_fwd": (ctypes.c_int, [_P, _I32, _P, _I32, _P, _P, _P] + [_I32] * 9 + [_P, _P, _P]),
    "tsplat_resize_bilinear_nhwc_fwd": (ctypes.c_int, [_P, _P] + [_I32] * 6 + [_P]),
    "tsplat_resize_bilinear_nchw_fwd": (ctypes.c_int, [_P, _P] + [_I32] * 5 + [_P]),
    "tsplat_upsample_bilinear_act_fwd": (ctypes.c_int, [_P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_conv2d_f32_nhwc_fwd": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P] + [_I32] * 7 + [_P]),
    "tsplat_residual_ln_fwd": (ctypes.c_int, [_P] * 5 + [ctypes.c_float, _P, _P, _I32, _I32, _P]),
    "tsplat_residual_ln_slabs_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, ctypes.c_float, _P, _P, _I32, _I32, _P]),
    "tsplat_gemm_x3_pack_bytes": (ctypes.c_size_t, [_I32, _I32]),
    "tsplat_gemm_x3_pack": (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    "tsplat_gemm_x3_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P]),
    "tsplat_residual_ln_bf16_fwd": (ctypes.c_int, [_P] * 5 + [ctypes.c_float, _P, _P, _I32, _I32, _P]),
    "tsplat_bias_act_fwd": (ctypes.c_int, [_P] * 4 + [_I32, _I32, ctypes.c_int64, _I32, _P]),
    "tsplat_bias_act_nhwc_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_int64, _I32, _I32, _P]),
    "tsplat_win_attn_partials_fwd": (ctypes.c_int, [_P] * 4 + [_I32] * 8 + [_P]),
    "tsplat_split_kv_bf16x3": (ctypes.c_int, [_P, _P, _P, ctypes.c_int64, _P]),
    "tsplat_linear_f32_split_x3_fwd": (ctypes.c_int, [_P, _I32, _P, _P, _P] + [_I32] * 4 + [_P]),
    "tsplat_win_attn_x3_fwd": (ctypes.c_int, [_P] * 4 + [_I32] * 7 + [_P]),
    "tsplat_win_attn_x3_partials_fwd": (ctypes.c_int, [_P] * 3 + [_I32] * 8 + [_P]),
    "tsplat_linear_f32_attn_merge_fwd": (ctypes.c_int, [_P] + [_I32] * 6 + [_P] * 3 + [ctypes.c_float, _P, _P, _I32,
                                                                                       _I32, _P]),
    "tsplat_linear_f32_fwd": (ctypes.c_int, [_P, _I32, _P, _I32] + [_P] * 4 + [ctypes.c_float, _P, _P, ctypes.c_int64]
                              + [_I32] * 3 + [_P]),
    "tsplat_wino_weight_floats": (ctypes.c_size_t, [_I32, _I32]),
    "tsplat_wino_weight_f32": (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    "tsplat_conv3x3_wino_f32_fwd": (ctypes.c_int, [_P, _P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_conv3x3_wino_cat_f32_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P] + [_I32] * 5 + [_P]),
    "tsplat_wino_weight_bf16x3_bytes": (ctypes.c_size_t, [_I32, _I32]),
    "tsplat_wino_weight_bf16x3": (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    "tsplat_conv3x3_wino_bf16x3_fwd": (ctypes.c_int, [_P, _P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_conv3x3_wino_bf16x3_cat_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P] + [_I32] * 5 + [_P]),
    "tsplat_conv3x3_wino_bf16x3_ex_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_conv3x3_few_form": (ctypes.c_int32, [_I32] * 5),
    "tsplat_conv3x3_few_bf16x3_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P] + [_I32] * 6 + [_P]),
    "tsplat_split_bf16x3": (ctypes.c_int, [_P, _P, ctypes.c_int64, _I32, _I32, _P]),
    "tsplat_conv2d_bf16_weight_bytes": (ctypes.c_size_t, [_I32, _I32, _I32]),
    "tsplat_conv2d_bf16_fwd": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P] + [_I32] * 7 + [_P]),
}

ERRORS = {-1: "invalid argument", -2: "HIP launch error"}


def lib_path() -> Path:
    return _LIB_PATH


def load(build_if_missing: bool = False):
    """Load the HIP library (torch must already be imported so its HIP runtime is the one used)."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        if build_if_missing:
            from .build import build

            build()
        else:
            raise RuntimeError(
                f"transplat HIP library not built ({_LIB_PATH}); run `python -m transplat_amd.build`"
            )
    lib = ctypes.CDLL(str(_LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if os.environ.get("TSPLAT_DEBUG", "0") == "1":  # every entry point: sync + check per launch
        lib.tsplat_set_debug(1)
    _lib = lib
    return lib


def debug_enabled() -> bool:
    """Whether tsplat_set_debug mode is on (it synchronises after every launch, which stream capture
    forbids: callers that capture a hipGraph refuse to while it is on)."""
    lib = load()
    was = lib.tsplat_set_debug(1)
    lib.tsplat_set_debug(was)
    return bool(was)


# routes.record() sets this to note every entry point a step calls (None otherwise)
ROUTE_HOOK = None


def check(status: int, what: str, route: str | None = None) -> None:
    """Raise on a non-zero C-ABI status. `route`: the arithmetic a flag selected for this call
    (noted by routes.record(), which derives the bench line's precision statement)."""
    if status != 0:
        raise RuntimeError(f"{what} failed: {ERRORS.get(status, status)}")
    if ROUTE_HOOK is not None:
        ROUTE_HOOK(what, route)


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("transplat HIP ops need device tensors (no CPU path)")
    return t.data_ptr()


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


PROF_IDS = {"raster_preprocess": 1, "raster_scan": 2, "raster_scatter": 3, "raster_render": 4,
            "uv_coarse": 5, "uv_cross": 6, "msda": 7, "win_attn": 8, "raster": 9,
            "group_norm": 10, "uv_cross_table": 11, "linear": 12, "mha": 13, "conv": 14, "wino_conv": 15,
            "gemm_x3": 16}


def prof_enable(name: str | None) -> None:
    check(load().tsplat_prof_enable(PROF_IDS[name] if name else 0), "tsplat_prof_enable")


def prof_read() -> tuple[float, int]:
    """(total ms, launches) of the kernel being timed since the last enable/read."""
    ms = ctypes.c_double(0.0)
    n = _I32(0)
    check(load().tsplat_prof_read(ctypes.byref(ms), ctypes.byref(n)), "tsplat_prof_read")
    return ms.value, n.value
