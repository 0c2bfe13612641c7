"""Python face of the encoder-side gfx950 kernels (C-ABI in include/transplat_hip.h).

Signatures match the CPU restatements in oracle/encoder_ops.py one for one. Every function
requires device tensors and the in-tree HIP library; there is no fallback path.
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _lib


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def small_inverse(x: torch.Tensor) -> torch.Tensor:
    """Inverse of [..., d, d] (d = 2, 3, 4) camera matrices. Device tensors: one HIP launch
    (tsplat_small_inverse) instead of rocsolver's getrf/getri chain. Host tensors (camera setup
    from host data, e.g. the CPU oracle path or dataset prep) use torch.linalg on the host."""
    if not x.is_cuda:
        return torch.linalg.inv_ex(x)[0]
    lib = _lib.load()
    d = x.shape[-1]
    xf = _f32(x)
    out = torch.empty_like(xf)
    n = xf.numel() // (d * d)
    _lib.check(lib.tsplat_small_inverse(_lib.ptr(xf), _lib.ptr(out), n, d, _lib.stream_ptr(x.device)),
               "tsplat_small_inverse")
    return out.to(x.dtype) if x.dtype != torch.float32 else out


def pack_cameras(intr: torch.Tensor, pose: torch.Tensor) -> torch.Tensor:
    """[N, 30] = K^-1, K, R, t per (v b) camera (the inputs of calculate_grid,
    reference depth_predictor_trans.py:36-49, with K^-1 taken by torch.inverse as there)."""
    intr = intr.float()
    return torch.cat(
        [small_inverse(intr).reshape(-1, 9), intr.reshape(-1, 9), pose[:, :3, :3].reshape(-1, 9).float(),
         pose[:, :3, 3].float()], dim=1).contiguous()


def window_attention(q, k, v, h: int, w: int, num_splits: int, with_shift: bool, kv_shift: int = 0):
    """Shifted-window attention (reference single_head_split_window_attention).
    q [B, L, C]; k, v [B, L, C] or [B, m, L, C] -> [B, L, C]. bf16 inputs (the dense layers under
    bf16 autocast) run the bf16-MFMA kernel and return bf16; everything else runs exact fp32.
    kv_shift: query batch i attends to the keys / values of batch (i + kv_shift) % B."""
    lib = _lib.load()
    b, l, c = q.shape
    m = 1 if k.dim() == 3 else k.shape[1]
    wl = (h // num_splits) * (w // num_splits)
    if q.dtype == k.dtype == v.dtype == torch.bfloat16 and wl % 128 == 0:
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty((b, l, c), dtype=torch.bfloat16, device=q.device)
        nbytes = int(lib.tsplat_win_attn_bf16_workspace_bytes(b, h, w, m, num_splits))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=q.device) if nbytes else None
        rc = lib.tsplat_win_attn_bf16_shift_fwd(_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(out), _lib.ptr(ws),
                                                b, h, w, c, m, num_splits, int(with_shift), int(kv_shift) % b,
                                                _lib.stream_ptr(q.device))
        _lib.check(rc, "tsplat_win_attn_bf16_shift_fwd")
        return out
    if kv_shift:
        k, v = torch.roll(k, -kv_shift, dims=0), torch.roll(v, -kv_shift, dims=0)
    q, k, v = _f32(q), _f32(k), _f32(v)
    out = torch.empty((b, l, c), dtype=torch.float32, device=q.device)
    nbytes = int(lib.tsplat_win_attn_workspace_bytes(b, h, w, m, num_splits))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=q.device) if nbytes else None
    rc = lib.tsplat_win_attn_fwd(_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(out), _lib.ptr(ws), b, h, w, c,
                                 m, num_splits, int(with_shift), _lib.stream_ptr(q.device))
    _lib.check(rc, "tsplat_win_attn_fwd")
    return out


def uv_coarse(feat, intr, pose, disp, h: int, w: int):
    """Coarse correlation volume. feat [B, 2, HW, C] -> [B*2, HW, D] (see oracle.uv_coarse)."""
    lib = _lib.load()
    b, _, hw, c = feat.shape
    d = disp.shape[1]
    feat = _f32(feat)
    cams = pack_cameras(intr, pose)
    disp = _f32(disp)
    out = torch.empty((b * 2, hw, d), dtype=torch.float32, device=feat.device)
    rc = lib.tsplat_uv_coarse_fwd(_lib.ptr(feat), _lib.ptr(cams), _lib.ptr(disp), _lib.ptr(out), b, h, w,
                                  c, d, _lib.stream_ptr(feat.device))
    _lib.check(rc, "tsplat_uv_coarse_fwd")
    return out


def uv_cross(value, key, intr, pose, disp, offsets, logits, h: int, w: int):
    """Fine cross correlation. value, key [B, 2, HW, C]; offsets [B*2, HW, D*P*2];
    logits [B*2, HW, D*P] -> [B*2, HW, D] (see oracle.uv_cross).

    Two steps: the correlation table G[(b v)] = key_v value_(1-v)^T [HW, HW] as one batched
    fp32 library GEMM (hipBLASLt, MFMA; autocast off so it stays fp32), then
    tsplat_uv_cross_table_fwd gathers 4 points x 4 bilinear corners of G per (pixel, depth)."""
    lib = _lib.load()
    b, _, hw, c = value.shape
    d = disp.shape[1]
    p = logits.shape[-1] // d
    if value.dtype == torch.bfloat16 and value.is_cuda and _UV_TABLE_BF16:
        # bf16 dense mode: value is a bf16 linear output, so value^T is exact in bf16 and the table
        # G = key value^T can run on bf16 MFMA with fp32 accumulation and output: key split as
        # key_hi + key_lo (two bf16 halves, residual error ~2^-17 relative) and both halves taken
        # in ONE GEMM with K = 2C ([key_hi | key_lo] x [value | value]^T)
        kf = _f32(key).reshape(b * 2, hw, c)
        k_hi = kf.to(torch.bfloat16)
        k2 = torch.cat((k_hi, (kf - k_hi.float()).to(torch.bfloat16)), dim=-1)
        vb = torch.flip(value, dims=[1]).reshape(b * 2, hw, c)
        with torch.autocast("cuda", enabled=False):
            table = torch.bmm(k2, torch.cat((vb, vb), dim=-1).transpose(1, 2), out_dtype=torch.float32)
        value = None
        key, offsets, logits, disp = map(_f32, (key, offsets, logits, disp))
    elif _DENSE == "bf16x3" and value.is_cuda and c % 4 == 0:
        # bf16x3 dense mode: the table in split-bf16 precision as ONE hipBLASLt bf16 GEMM with K = 3C,
        # [key_hi | key_hi | key_lo] x [val_hi | val_lo | val_hi]^T, fp32 output (47 vs 83 us for the
        # fp32 bmm at b = 1, and vs 104 us on tsplat_linear_bf16x3_fwd, profiles/r4/split_gemm2.log;
        # <= 3 * 2^-18 relative per product)
        value, key, offsets, logits, disp = map(_f32, (value, key, offsets, logits, disp))
        k3 = split_bf16x3(key.reshape(b * 2, hw, c))
        v3 = split_bf16x3(torch.flip(value, dims=[1]).reshape(b * 2, hw, c), weight_order=True)
        with torch.autocast("cuda", enabled=False):
            table = torch.bmm(k3, v3.transpose(1, 2), out_dtype=torch.float32)
    else:
        value, key, offsets, logits, disp = map(_f32, (value, key, offsets, logits, disp))
        with torch.autocast("cuda", enabled=False):
            table = torch.bmm(key.reshape(b * 2, hw, c),
                              torch.flip(value, dims=[1]).reshape(b * 2, hw, c).transpose(1, 2))
    cams = pack_cameras(intr, pose)
    out = torch.empty((b * 2, hw, d), dtype=torch.float32, device=table.device)
    rc = lib.tsplat_uv_cross_table_fwd(_lib.ptr(table), _lib.ptr(cams), _lib.ptr(disp), _lib.ptr(offsets),
                                       _lib.ptr(logits), _lib.ptr(out), b, h, w, c, d, p, _lib.stream_ptr(table.device))
    _lib.check(rc, "tsplat_uv_cross_table_fwd")
    return out


def uv_cross_direct(value, key, intr, pose, disp, offsets, logits, h: int, w: int):
    """The same op in one gather kernel without the table (tsplat_uv_cross_fwd: 16 feature-row
    samples per (pixel, depth)); kept as the table-free variant (no [HW, HW] buffer)."""
    lib = _lib.load()
    b, _, hw, c = value.shape
    d = disp.shape[1]
    p = logits.shape[-1] // d
    value, key, offsets, logits, disp = map(_f32, (value, key, offsets, logits, disp))
    cams = pack_cameras(intr, pose)
    out = torch.empty((b * 2, hw, d), dtype=torch.float32, device=value.device)
    rc = lib.tsplat_uv_cross_fwd(_lib.ptr(value), _lib.ptr(key), _lib.ptr(cams), _lib.ptr(disp),
                                 _lib.ptr(offsets), _lib.ptr(logits), _lib.ptr(out), b, h, w, c, d, p,
                                 _lib.stream_ptr(value.device))
    _lib.check(rc, "tsplat_uv_cross_fwd")
    return out


def ms_deform_attn(value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                   im2col_step: int = 64):
    """mmcv ext_module.ms_deform_attn_forward (tsplat_ms_deform_attn_fwd): value [bs, keys, heads, hd],
    spatial shapes [L, 2] / level starts [L] (int64), sampling_locations [bs, nq, heads, L, P, 2],
    attention_weights [bs, nq, heads, L, P] -> [bs, nq, heads * hd] fp32. Raises, as mmcv's
    assertion does, when min(bs, im2col_step) does not divide bs."""
    lib = _lib.load()
    bs, nk, nh, hd = value.shape
    _, nq, nh2, nl, npt, two = sampling_locations.shape
    if nh2 != nh or two != 2 or tuple(attention_weights.shape) != (bs, nq, nh, nl, npt):
        raise ValueError("sampling_locations / attention_weights do not match value's heads")
    shapes = value_spatial_shapes.to(device=value.device, dtype=torch.int64).contiguous()
    starts = value_level_start_index.to(device=value.device, dtype=torch.int64).contiguous()
    if tuple(shapes.shape) != (nl, 2) or tuple(starts.shape) != (nl,):
        raise ValueError(f"spatial shapes {tuple(shapes.shape)} / level starts {tuple(starts.shape)} != {nl} levels")
    out = torch.empty((bs, nq, nh * hd), dtype=torch.float32, device=value.device)
    rc = lib.tsplat_ms_deform_attn_fwd(_lib.ptr(_f32(value)), _lib.ptr(shapes), _lib.ptr(starts),
                                       _lib.ptr(_f32(sampling_locations)), _lib.ptr(_f32(attention_weights)),
                                       _lib.ptr(out), bs, nk, nh, hd, nl, nq, npt, int(im2col_step),
                                       _lib.stream_ptr(value.device))
    _lib.check(rc, "tsplat_ms_deform_attn_fwd")
    return out


def msda(value, loc, weights, h: int, w: int):
    """Single-level single-head deformable sampling. value [N, HW, C], loc [N, Q, P, 2],
    weights [N, Q, P] -> [N, Q, C] (see oracle.msda)."""
    lib = _lib.load()
    n, hw, c = value.shape
    _, q, p, _ = loc.shape
    value, loc, weights = _f32(value), _f32(loc), _f32(weights)
    out = torch.empty((n, q, c), dtype=torch.float32, device=value.device)
    rc = lib.tsplat_msda_fwd(_lib.ptr(value), _lib.ptr(loc), _lib.ptr(weights), _lib.ptr(out), n, h, w, c,
                             q, p, _lib.stream_ptr(value.device))
    _lib.check(rc, "tsplat_msda_fwd")
    return out


def msda_raw(value, ow, points: int, h: int, w: int):
    """msda(value, ref_2d + off / (w, h), softmax(logits), h, w) from the raw [N, h w, >= 3 points]
    rows ow = [offsets (dx, dy) x points | logits x points | ...] (tsplat_msda_raw_fwd; see
    oracle.msda_raw). value [N, h w, 128] -> [N, h w, 128]."""
    lib = _lib.load()
    n, hw, c = value.shape
    value, ow = _f32(value), _f32(ow)
    if ow.shape[:2] != (n, hw) or ow.shape[-1] < 3 * points or not ow.is_contiguous():
        raise ValueError(f"ow {tuple(ow.shape)} does not match value {tuple(value.shape)} / {points} points")
    out = torch.empty((n, hw, c), dtype=torch.float32, device=value.device)
    rc = lib.tsplat_msda_raw_fwd(_lib.ptr(value), _lib.ptr(ow), _lib.ptr(out), n, h, w, c, points, ow.shape[-1],
                                 _lib.stream_ptr(value.device))
    _lib.check(rc, "tsplat_msda_raw_fwd")
    return out


def adapter_cameras(extrinsics: torch.Tensor, intrinsics: torch.Tensor, image_shape) -> torch.Tensor:
    """[N, 22] per-camera constants of tsplat_gaussian_adapter_fwd: c2w R, c2w t, K^-1 of the
    normalised intrinsics, and the scale multiplier of GaussianAdapter.get_scale_multiplier
    (reference gaussian_adapter.py:98-109). Inverses via inv_ex (no host sync)."""
    h, w = image_shape
    ext = extrinsics.reshape(-1, 4, 4).float()
    k = intrinsics.reshape(-1, 3, 3).float()
    kinv = small_inverse(k)
    k2inv = small_inverse(k[:, :2, :2].contiguous())
    pix = torch.stack([torch.full_like(k[:, 0, 0], 1.0 / w), torch.full_like(k[:, 0, 0], 1.0 / h)], -1)
    mult = 0.1 * (k2inv @ pix[..., None])[..., 0].sum(-1)
    return torch.cat([ext[:, :3, :3].reshape(-1, 9), ext[:, :3, 3], kinv.reshape(-1, 9), mult[:, None]], 1).contiguous()


_ACTS = {"none": 0, "silu": 1, "gelu": 2, "relu": 3}
_AFFINE_ID: dict = {}


_NO_CONV_EPI = os.environ.get("TSPLAT_NO_CONV_EPI", "")  # A/B timing knob only: "all" or a site name


def conv_bias_act(conv, x, act: str = "none", residual=None, site: str = "", extra=()):
    """conv(x) + bias -> act [-> + residual (-> relu for "relu")] with the bias, activation and
    residual in ONE pass after the bias-free MIOpen convolution (tsplat_bias_act_fwd). Under bf16
    autocast (config C3's dense layers) or for outputs the kernel's float4 layout cannot take, the
    module's own forward and PyTorch activations run instead (dense-layer glue, same math).
    Used on the depth predictor's full-resolution conv -> GELU -> conv heads (+0.4 % e2e); on the
    DPT ResidualConvUnits the bias-free convolutions measured 3 % slower end to end (A/B with
    TSPLAT_NO_CONV_EPI=<site>), so those keep the module path."""
    import torch.nn.functional as F

    if not x.is_cuda:
        raise RuntimeError("transplat HIP ops need device tensors (no CPU path)")
    if (residual is None and act in _ACTS and _NO_CONV_EPI not in ("all", site)
            and getattr(conv, "padding_mode", "zeros") == "zeros"
            and conv_bf16_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, extra)):
        return conv_bf16(x, conv.weight, conv.bias, act, extra)  # bf16 autocast: bias + act fused
    fused = (not torch.is_autocast_enabled("cuda") and x.dtype == torch.float32 and _NO_CONV_EPI not in ("all", site)
             and getattr(conv, "padding_mode", "zeros") == "zeros")
    if (fused and residual is None and act in _WINO_ACT
            and conv3x3_wino_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, extra,
                                vs_miopen=True)):
        # the Winograd kernel reads the concatenation in place and applies the bias and the
        # activation in its epilogue
        return conv3x3_wino(x, conv.weight, conv.bias, act, extra)
    if extra:
        x = torch.cat([x, *extra], dim=1)
    if fused:
        y = conv2d_fallback(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
        # the kernel indexes the residual with y's NCHW layout: a broadcastable residual ([C, 1, 1],
        # a batch-1 map) takes the module path, where `y + residual` broadcasts
        fused = ((y.shape[-1] * y.shape[-2]) % 4 == 0 and y.is_contiguous()
                 and (residual is None or tuple(residual.shape) == tuple(y.shape)))
    if not fused:
        y = conv(x)
        if act == "gelu":
            y = F.gelu(y)
        elif act == "relu":
            y = torch.relu(y)
        if residual is not None:
            y = y + residual
            if act == "relu":
                y = torch.relu(y)
        return y
    lib = _lib.load()
    n, c = y.shape[:2]
    res = _f32(residual) if residual is not None else None
    rc = lib.tsplat_bias_act_fwd(_lib.ptr(y), _lib.ptr(conv.bias), _lib.ptr(res), _lib.ptr(y), n, c,
                                 y.shape[-1] * y.shape[-2], _ACTS[act], _lib.stream_ptr(y.device))
    _lib.check(rc, "tsplat_bias_act_fwd")
    return y


def instance_norm(x, eps: float, act: str = "none", residual=None):
    """InstanceNorm2d (affine=False, instance statistics) as GroupNorm with one group per channel
    (tsplat_group_norm_fwd), with "relu" and the ResidualBlock ending relu(residual + relu(norm))."""
    c = x.shape[1]
    key = (c, x.device)
    if key not in _AFFINE_ID:
        _AFFINE_ID[key] = (torch.ones(c, device=x.device), torch.zeros(c, device=x.device))
    w, b = _AFFINE_ID[key]
    return group_norm(x, c, w, b, eps, act, residual)


_BF16_NORMS = os.environ.get("TSPLAT_BF16_NORMS", "1") != "0"  # A/B knob: bf16-I/O norm kernels (C3)
_CAT_RES = os.environ.get("TSPLAT_GN_CAT_RES", "1") != "0"  # A/B knob: concatenated residuals read in place
BF16_NORMS = _BF16_NORMS
_UV_TABLE_BF16 = os.environ.get("TSPLAT_UV_TABLE_BF16", "1") != "0"  # A/B knob: split-bf16 table GEMM (C3)


def group_norm(x, num_groups: int, weight, bias, eps: float, act: str = "none", residual=None, pre_bias=None):
    """act(GroupNorm(x + pre_bias)) [+ residual] over [N, C, *spatial] (see tsplat_group_norm_fwd);
    pre_bias is the bias of a convolution that ran without it. A bf16 x (bf16 dense mode) is read
    and the result written in bf16 (tsplat_group_norm_bf16_fwd, fp32 statistics), else fp32.
    residual may be a pair (r1, r2): the channel concatenation cat([r1, r2], 1), read in place by
    the fp32 kernel (tsplat_group_norm_cat_res_fwd)."""
    lib = _lib.load()
    n, c = x.shape[:2]
    hw = x[0, 0].numel()
    if isinstance(residual, (tuple, list)):
        r1, r2 = residual
        if not (_CAT_RES and x.dtype == torch.float32 and r1.dtype == r2.dtype == torch.float32 and x.is_cuda):
            return group_norm(x, num_groups, weight, bias, eps, act, torch.cat([r1, r2], dim=1), pre_bias)
        r1, r2 = r1.contiguous(), r2.contiguous()
        if (r1.shape[0] != n or r2.shape[0] != n or r1.shape[1] + r2.shape[1] != c or r1.shape[2:] != x.shape[2:]
                or r2.shape[2:] != x.shape[2:]):
            raise ValueError(f"residual parts {tuple(r1.shape)} + {tuple(r2.shape)} != input {tuple(x.shape)}")
        xf = _f32(x)
        y = torch.empty_like(xf)
        ws = torch.empty(int(lib.tsplat_group_norm_workspace_bytes(n, c, hw, num_groups)), dtype=torch.uint8,
                         device=x.device)
        pb = _f32(pre_bias) if pre_bias is not None else None
        rc = lib.tsplat_group_norm_cat_res_fwd(_lib.ptr(xf), _lib.ptr(pb), _lib.ptr(_f32(weight)),
                                               _lib.ptr(_f32(bias)), _lib.ptr(r1), _lib.ptr(r2), r1.shape[1],
                                               _lib.ptr(y), _lib.ptr(ws), n, c, hw, num_groups, float(eps),
                                               _ACTS[act], _lib.stream_ptr(x.device))
        _lib.check(rc, "tsplat_group_norm_cat_res_fwd")
        return y
    if x.dtype == torch.bfloat16 and x.is_cuda and _BF16_NORMS:
        if residual is not None and residual.dtype != torch.bfloat16:
            # the module path rounds the norm's output to bf16 (GroupNorm32 casts back to x's dtype)
            # and then promotes bf16 + fp32 to fp32: keep the fp32 residual stream un-narrowed
            return group_norm(x, num_groups, weight, bias, eps, act, None, pre_bias).float() + residual
        xb = x.contiguous()
        res = residual.contiguous() if residual is not None else None
        if res is not None and res.shape != x.shape:
            raise ValueError(f"residual {tuple(res.shape)} != input {tuple(x.shape)}")
        y = torch.empty_like(xb)
        ws = torch.empty(int(lib.tsplat_group_norm_workspace_bytes(n, c, hw, num_groups)), dtype=torch.uint8,
                         device=x.device)
        pb = _f32(pre_bias) if pre_bias is not None else None
        rc = lib.tsplat_group_norm_bf16_fwd(_lib.ptr(xb), _lib.ptr(pb), _lib.ptr(_f32(weight)), _lib.ptr(_f32(bias)),
                                            _lib.ptr(res) if res is not None else None, _lib.ptr(y), _lib.ptr(ws),
                                            n, c, hw, num_groups, float(eps), _ACTS[act], _lib.stream_ptr(x.device))
        _lib.check(rc, "tsplat_group_norm_bf16_fwd")
        return y
    xf = _f32(x)
    res = _f32(residual) if residual is not None else None
    if res is not None and res.shape != x.shape:
        raise ValueError(f"residual {tuple(res.shape)} != input {tuple(x.shape)}")
    y = torch.empty_like(xf)
    ws = torch.empty(int(lib.tsplat_group_norm_workspace_bytes(n, c, hw, num_groups)), dtype=torch.uint8,
                     device=x.device)
    pb = _f32(pre_bias) if pre_bias is not None else None
    rc = lib.tsplat_group_norm_fwd(_lib.ptr(xf), _lib.ptr(pb), _lib.ptr(_f32(weight)), _lib.ptr(_f32(bias)),
                                   _lib.ptr(res) if res is not None else None, _lib.ptr(y), _lib.ptr(ws), n, c, hw,
                                   num_groups, float(eps), _ACTS[act], _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_group_norm_fwd")
    return y


_LIN_GELU, _LIN_LN, _LIN_RES, _LIN_SPLIT, _LIN_BIAS, _LIN_GELU_IN = 1, 2, 4, 8, 16, 32
_LIN_RES_PRE_LN, _LIN_RELU_IN, _LIN_BF16X3, _LIN_X_BF16, _LIN_OUT_BF16 = 64, 128, 256, 512, 1024
# the fused transformer linears' products in bf16x3 inside dense_precision("bf16x3") (the kernel's
# split-bf16 form, flag 256); TSPLAT_LINF3=0 keeps them exact fp32 in that mode
_LINF3 = os.environ.get("TSPLAT_LINF3", "1") == "1"


def _lin_precision_flag() -> int:
    return _LIN_BF16X3 if _LINF3 and _DENSE == "bf16x3" else 0


def _lin_route(flags: int) -> str:
    """The arithmetic of a tsplat_linear_f32_* call with these flags (routes.record)."""
    r = "bf16x3" if flags & _LIN_BF16X3 else "exact fp32"
    return r + (", bf16 I/O" if flags & (_LIN_X_BF16 | _LIN_OUT_BF16) else "")


def fused_linear(x1, weight, x2=None, bias=None, gelu: bool = False, ln=None, residual=None, split: bool = False,
                 gelu_in: bool = False, relu_in: bool = False, res_pre_ln: bool = False, out_dtype=torch.float32):
    """epilogue([x1 | x2] weight^T) in one exact-fp32 MFMA launch (tsplat_linear_f32_fwd; bf16x3
    products inside dense_precision("bf16x3"), see _LINF3):
    (+ bias) -> (exact GELU) -> (LayerNorm with ln = (gamma, beta, eps), N = 128) -> (+ residual);
    gelu_in / relu_in apply exact GELU / ReLU to the input first (the producing layer's activation,
    N = 128); res_pre_ln adds the residual before the LayerNorm (post-norm: LN(y + residual)).
    x1 [..., k1], x2 [..., k2] (concatenated along the last axis without materialising it);
    split=True returns the N / 128 column blocks as separate contiguous [..., 128] tensors. A bf16 x1
    (no x2) is read as bf16 and widened exactly in the kernel; out_dtype=torch.bfloat16 writes the
    output in bf16 (no residual) -- the bf16 window attention's operands / message without casts."""
    lib = _lib.load()
    lead = x1.shape[:-1]
    k1 = x1.shape[-1]
    k2 = x2.shape[-1] if x2 is not None else 0
    n = weight.shape[0]
    if weight.shape[1] != k1 + k2:
        raise ValueError(f"weight {tuple(weight.shape)} does not match k1 + k2 = {k1 + k2}")
    xbf = x1.dtype == torch.bfloat16 and x2 is None and x1.is_cuda
    if out_dtype not in (torch.float32, torch.bfloat16) or (out_dtype == torch.bfloat16 and residual is not None):
        raise ValueError(f"out_dtype {out_dtype} (with residual={residual is not None}) not supported")
    a = (x1.contiguous() if xbf else _f32(x1)).reshape(-1, k1)
    m = a.shape[0]
    b = _f32(x2).reshape(-1, k2) if x2 is not None else None
    if b is not None and b.shape[0] != m:
        raise ValueError("x1 and x2 row counts differ")
    flags = (_LIN_GELU if gelu else 0) | (_LIN_LN if ln is not None else 0) | (_LIN_BIAS if bias is not None else 0)
    flags |= (_LIN_GELU_IN if gelu_in else 0) | (_LIN_RELU_IN if relu_in else 0)
    flags |= _LIN_RES_PRE_LN if res_pre_ln and residual is not None else 0
    flags |= _lin_precision_flag()
    flags |= (_LIN_X_BF16 if xbf else 0) | (_LIN_OUT_BF16 if out_dtype == torch.bfloat16 else 0)
    res = None
    if residual is not None:
        res = _f32(residual).reshape(m, n)
        flags |= _LIN_RES
    if split:
        flags |= _LIN_SPLIT
        out = torch.empty((n // 128, m, 128), dtype=out_dtype, device=x1.device)
    else:
        out = torch.empty((m, n), dtype=out_dtype, device=x1.device)
    g, bt, eps = (_f32(ln[0]), _f32(ln[1]), float(ln[2])) if ln is not None else (None, None, 0.0)
    bb = _f32(bias) if bias is not None else None
    rc = lib.tsplat_linear_f32_fwd(_lib.ptr(a), k1, _lib.ptr(b), k2, _lib.ptr(_f32(weight)), _lib.ptr(bb),
                                   _lib.ptr(g), _lib.ptr(bt), eps, _lib.ptr(res), _lib.ptr(out), m * 128, m, n,
                                   flags, _lib.stream_ptr(x1.device))
    _lib.check(rc, "tsplat_linear_f32_fwd", _lin_route(flags))
    if split:
        return [t.reshape(*lead, 128) for t in out.unbind(0)]
    return out.reshape(*lead, n)


# bf16x3 window attention (tsplat_win_attn_x3_*) as the "auto" attention of the bf16x3 dense mode
# (see auto_attention); TSPLAT_ATTN_X3=0 keeps the exact-fp32 kernel in that mode
_ATTN_X3 = os.environ.get("TSPLAT_ATTN_X3", "1") == "1"


def split_kv_bf16x3(k, v):
    """[kh | kl | vh | vl] bf16 (x = xh + xl) of two same-shape fp32 tensors, one launch."""
    lib = _lib.load()
    k, v = _f32(k).contiguous(), _f32(v).contiguous()
    if k.shape != v.shape:
        raise ValueError(f"k {tuple(k.shape)} and v {tuple(v.shape)} differ")
    out = torch.empty((4, k.numel()), dtype=torch.bfloat16, device=k.device)
    _lib.check(lib.tsplat_split_kv_bf16x3(_lib.ptr(k), _lib.ptr(v), _lib.ptr(out), k.numel(),
                                          _lib.stream_ptr(k.device)), "tsplat_split_kv_bf16x3")
    return out


def window_attention_x3(q, k, v, h: int, w: int, num_splits: int, with_shift: bool):
    """window_attention(q, k, v) (fp32 [B, HW, 128], one key view) in bf16x3 precision
    (tsplat_win_attn_x3_fwd: split-bf16 products on bf16 MFMA, fp32 softmax)."""
    lib = _lib.load()
    b, l, c = q.shape
    m = 1 if k.dim() == 3 else k.shape[1]
    kv = split_kv_bf16x3(k, v)
    qf = _f32(q).contiguous()
    out = torch.empty_like(qf)
    ws = torch.empty(max(int(lib.tsplat_win_attn_workspace_bytes(b, h, w, m, num_splits)), 4), dtype=torch.uint8,
                     device=q.device)
    _lib.check(lib.tsplat_win_attn_x3_fwd(_lib.ptr(qf), _lib.ptr(kv), _lib.ptr(out), _lib.ptr(ws), b, h, w, c, m,
                                          num_splits, int(with_shift), _lib.stream_ptr(q.device)),
               "tsplat_win_attn_x3_fwd")
    return out


def attention_x3_ready(b: int, h: int, w: int, m: int, num_splits: int) -> bool:
    """True when attention_merge runs the bf16x3 kernel for this shape (the x3 precision is active
    and the launch splits the keys), i.e. when the k / v projection may hand it pre-split operands
    (linear_kv_x3) instead of fp32 k / v."""
    return _ATTN == "bf16x3" and int(_lib.load().tsplat_win_attn_split(b, h, w, m, num_splits)) > 1


def linear_kv_x3(x, weight, x3_from: int):
    """[x W^T] column blocks of 128 (the q | k | v or k | v projection): blocks before x3_from as fp32
    [..., 128] tensors, the rest as ONE [kh | kl | vh | vl] bf16 buffer (tsplat_linear_f32_split_x3_fwd;
    bf16x3 products inside dense_precision("bf16x3")). Returns (list of fp32 blocks, kv_x3)."""
    lib = _lib.load()
    lead = x.shape[:-1]
    k1, n = x.shape[-1], weight.shape[0]
    a = _f32(x).reshape(-1, k1)
    m = a.shape[0]
    nb = n // 128
    out = torch.empty((x3_from, m, 128), dtype=torch.float32, device=x.device) if x3_from else None
    kv = torch.empty((2 * (nb - x3_from), m * 128), dtype=torch.bfloat16, device=x.device)
    _lib.check(lib.tsplat_linear_f32_split_x3_fwd(_lib.ptr(a), k1, _lib.ptr(_f32(weight)), _lib.ptr(out), _lib.ptr(kv), m,
                                                  n, x3_from, _lin_precision_flag(), _lib.stream_ptr(x.device)),
               "tsplat_linear_f32_split_x3_fwd", _lin_route(_lin_precision_flag()))
    blocks = [t.reshape(*lead, 128) for t in out.unbind(0)] if out is not None else []
    return blocks, kv


def attention_merge(q, k, v, h: int, w: int, num_splits: int, with_shift: bool, merge_weight, ln, residual=None,
                    kv_shift: int = 0, kv_x3=None, kv_views: int = 1):
    """norm(window_attention(q, k, v) merge_weight^T) [+ residual] for the fp32 transformer layer.
    Where the attention kernel splits the keys (b = 1 at 64x64), the combine of its partials runs
    in the merge kernel's operand staging (tsplat_win_attn_partials_fwd +
    tsplat_linear_f32_attn_merge_fwd: no combine launch, no [B, L, 128] attention output);
    otherwise window_attention + fused_linear. kv_shift: query batch i attends to the keys /
    values of batch (i + kv_shift) % B (the two-view cross pairing without a swapped copy). kv_x3:
    the bf16x3 kernel's pre-split [kh | kl | vh | vl] operand (linear_kv_x3) in place of k / v
    (None), for shapes where attention_x3_ready() holds; kv_views = the key views per query batch it
    holds ([4, B * kv_views * L * 128], i.e. k / v of shape [B, kv_views, L, 128])."""
    lib = _lib.load()
    b, l, c = q.shape
    if kv_x3 is not None:
        if not attention_x3_ready(b, h, w, kv_views, num_splits):
            raise ValueError("kv_x3 given for a shape / precision that does not run the bf16x3 kernel")
        if kv_x3.numel() != 4 * b * kv_views * l * c:
            raise ValueError(f"kv_x3 holds {kv_x3.numel()} values, not 4 x {b} x {kv_views} key views x {l} x {c}")
        return _merge_partials(lib, q, None, None, h, w, num_splits, with_shift, merge_weight, ln, residual,
                               kv_shift, kv_views, kv_x3)
    m = 1 if k.dim() == 3 else k.shape[1]
    fp32 = q.dtype == k.dtype == v.dtype == torch.float32
    wl = (h // num_splits) * (w // num_splits)
    if attention_bf16_ready(h, w, num_splits):
        # bf16 attention (config C3): the projections' outputs in bf16 (attention_bf16_ready lets the
        # layer ask fused_linear for them; fp32 ones are rounded here), the bf16 MFMA kernel with the
        # cross pairing as a key-batch shift, the bf16 message widened by the merge projection's load
        qb, kb, vb = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
        if not _BF16IO and kv_shift:
            kb, vb = torch.roll(kb, -kv_shift, dims=0), torch.roll(vb, -kv_shift, dims=0)
            kv_shift = 0
        msg = window_attention(qb, kb, vb, h, w, num_splits, with_shift, kv_shift=kv_shift)
        return fused_linear(msg if _BF16IO else msg.float(), merge_weight, ln=ln, residual=residual)
    ks = int(lib.tsplat_win_attn_split(b, h, w, m, num_splits)) if fp32 and c == 128 else 0
    if ks <= 1:
        if kv_shift:
            k, v = torch.roll(k, -kv_shift, dims=0), torch.roll(v, -kv_shift, dims=0)
        msg = window_attention(q, k, v, h, w, num_splits, with_shift)
        return fused_linear(msg, merge_weight, ln=ln, residual=residual)
    return _merge_partials(lib, q, k, v, h, w, num_splits, with_shift, merge_weight, ln, residual, kv_shift, m, None)


# bf16 operands / outputs of the fused linear and the key-batch shift of the bf16 attention instead of
# cast / roll launches around them (C3 as stated); TSPLAT_LIN_BF16IO=0 restores the casts (A/B knob)
_BF16IO = os.environ.get("TSPLAT_LIN_BF16IO", "1") == "1"


def attention_bf16_ready(h: int, w: int, num_splits: int) -> bool:
    """True when attention_merge runs the bf16 window attention for this window shape (attention
    precision "bf16", window pixels a multiple of 128): the layer's q / k / v projections may then
    be written in bf16 directly (fused_linear out_dtype)."""
    return _ATTN == "bf16" and ((h // num_splits) * (w // num_splits)) % 128 == 0


def projections_bf16(h: int, w: int, num_splits: int) -> bool:
    """True when a transformer layer should ask fused_linear for bf16 q / k / v (see _BF16IO)."""
    return _BF16IO and attention_bf16_ready(h, w, num_splits)


def _merge_partials(lib, q, k, v, h, w, num_splits, with_shift, merge_weight, ln, residual, kv_shift, m, kv_x3):
    """attention_merge's key-split path: the attention kernel's partials + the merge projection."""
    b, l, c = q.shape
    q = q.contiguous()
    ws = torch.empty(int(lib.tsplat_win_attn_workspace_bytes(b, h, w, m, num_splits)), dtype=torch.uint8,
                     device=q.device)
    if _ATTN == "bf16x3":
        kv = kv_x3 if kv_x3 is not None else split_kv_bf16x3(k, v)
        rc = lib.tsplat_win_attn_x3_partials_fwd(_lib.ptr(q), _lib.ptr(kv), _lib.ptr(ws), b, h, w, c, m, num_splits,
                                                 int(with_shift), int(kv_shift), _lib.stream_ptr(q.device))
        _lib.check(rc, "tsplat_win_attn_x3_partials_fwd")
    else:
        k, v = k.contiguous(), v.contiguous()
        rc = lib.tsplat_win_attn_partials_fwd(_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(ws), b, h, w, c, m,
                                              num_splits, int(with_shift), int(kv_shift), _lib.stream_ptr(q.device))
        _lib.check(rc, "tsplat_win_attn_partials_fwd")
    n = merge_weight.shape[0]
    out = torch.empty((b, l, n), dtype=torch.float32, device=q.device)
    flags = (_LIN_LN if ln is not None else 0) | _lin_precision_flag()
    res = None
    if residual is not None:
        res = _f32(residual)
        flags |= _LIN_RES
    g, bt, eps = (_f32(ln[0]), _f32(ln[1]), float(ln[2])) if ln is not None else (None, None, 0.0)
    rc = lib.tsplat_linear_f32_attn_merge_fwd(_lib.ptr(ws), b, h, w, m, num_splits, int(with_shift),
                                              _lib.ptr(_f32(merge_weight)), _lib.ptr(g), _lib.ptr(bt), eps,
                                              _lib.ptr(res), _lib.ptr(out), n, flags, _lib.stream_ptr(q.device))
    _lib.check(rc, "tsplat_linear_f32_attn_merge_fwd", _lin_route(flags))
    return out


def residual_ln(x, y, ls, norm, bf16_out: bool = False):
    """(x + ls * y, LayerNorm(x + ls * y)) in one pass (tsplat_residual_ln_fwd); y None: (x, LN(x)).
    norm: an nn.LayerNorm (weight, bias, eps); ls: LayerScale gamma or None. A bf16 y, or
    bf16_out, selects the bf16 form (y read and LN written in bf16; x fp32 either way). y with one
    leading dimension more than x is the split-K slabs of gemm_x3 (summed in order,
    tsplat_residual_ln_slabs_fwd)."""
    lib = _lib.load()
    d = x.shape[-1]
    xf = _f32(x)
    rows = xf.numel() // d
    if y is not None and y.dim() == x.dim() + 1:
        if y.dtype != torch.float32 or bf16_out or tuple(y.shape[1:]) != tuple(x.shape):
            raise ValueError(f"residual_ln: slabs {tuple(y.shape)} for x {tuple(x.shape)}")
        yf = y.contiguous()
        x_out, n_out = torch.empty_like(xf), torch.empty_like(xf)
        rc = lib.tsplat_residual_ln_slabs_fwd(_lib.ptr(xf), _lib.ptr(yf), y.shape[0],
                                              _lib.ptr(_f32(ls)) if ls is not None else None,
                                              _lib.ptr(_f32(norm.weight)), _lib.ptr(_f32(norm.bias)), float(norm.eps),
                                              _lib.ptr(x_out), _lib.ptr(n_out), rows, d, _lib.stream_ptr(x.device))
        _lib.check(rc, "tsplat_residual_ln_slabs_fwd")
        return x_out, n_out
    if _BF16_NORMS and (bf16_out or (y is not None and y.dtype == torch.bfloat16)):
        yb = y.to(torch.bfloat16).contiguous() if y is not None else None
        x_out = torch.empty_like(xf) if y is not None else xf
        n_out = torch.empty(xf.shape, dtype=torch.bfloat16, device=xf.device)
        rc = lib.tsplat_residual_ln_bf16_fwd(_lib.ptr(xf), _lib.ptr(yb), _lib.ptr(_f32(ls)) if ls is not None else None,
                                             _lib.ptr(_f32(norm.weight)), _lib.ptr(_f32(norm.bias)), float(norm.eps),
                                             _lib.ptr(x_out) if y is not None else None, _lib.ptr(n_out), rows, d,
                                             _lib.stream_ptr(x.device))
        _lib.check(rc, "tsplat_residual_ln_bf16_fwd")
        return x_out, n_out
    yf = _f32(y) if y is not None else None
    x_out = torch.empty_like(xf) if y is not None else xf
    n_out = torch.empty_like(xf)
    rc = lib.tsplat_residual_ln_fwd(_lib.ptr(xf), _lib.ptr(yf), _lib.ptr(_f32(ls)) if ls is not None else None,
                                    _lib.ptr(_f32(norm.weight)), _lib.ptr(_f32(norm.bias)), float(norm.eps),
                                    _lib.ptr(x_out) if y is not None else None, _lib.ptr(n_out), rows, d,
                                    _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_residual_ln_fwd")
    return x_out, n_out


def layer_norm128(y, norm, residual=None, out_dtype=None):
    """[residual +] LayerNorm(y) over rows of 128 (tsplat_layer_norm128_fwd); y fp32 or bf16,
    residual fp32 (or None), output in out_dtype (default y's dtype)."""
    lib = _lib.load()
    if y.shape[-1] != 128:
        raise ValueError("layer_norm128: last dim must be 128")
    yc = y.contiguous() if y.dtype == torch.bfloat16 else _f32(y)
    out_dtype = out_dtype or yc.dtype
    res = _f32(residual) if residual is not None else None
    if res is not None and res.shape != y.shape:
        raise ValueError(f"residual {tuple(res.shape)} != {tuple(y.shape)}")
    out = torch.empty(y.shape, dtype=out_dtype, device=y.device)
    rc = lib.tsplat_layer_norm128_fwd(_lib.ptr(yc), int(yc.dtype == torch.bfloat16), _lib.ptr(res),
                                      _lib.ptr(_f32(norm.weight)), _lib.ptr(_f32(norm.bias)), float(norm.eps),
                                      _lib.ptr(out), int(out_dtype == torch.bfloat16), yc.numel() // 128,
                                      _lib.stream_ptr(y.device))
    _lib.check(rc, "tsplat_layer_norm128_fwd", "bf16 I/O, fp32 statistics" if yc.dtype == torch.bfloat16 else "fp32")
    return out


def depth_softmax(logits, disp):
    """(coarse disparity, max pdf) of softmax(logits, dim=1) over the depth candidates:
    logits [N, D, H, W], disp [N, D(, 1, 1)] -> two [N, 1, H, W] maps (tsplat_depth_softmax_fwd)."""
    lib = _lib.load()
    n, d, h, w = logits.shape
    lf = _f32(logits)
    df = _f32(disp.reshape(n, d))
    coarse = torch.empty((n, 1, h, w), dtype=torch.float32, device=logits.device)
    pmax = torch.empty_like(coarse)
    _lib.check(lib.tsplat_depth_softmax_fwd(_lib.ptr(lf), _lib.ptr(df), _lib.ptr(coarse), _lib.ptr(pmax), n, d,
                                            h * w, _lib.stream_ptr(logits.device)), "tsplat_depth_softmax_fwd")
    return coarse, pmax


def depth_tail(fullres, head, near, far):
    """(depths, densities) of the depth head tail: fullres [(v b), 1, h, w], head [(v b), 2, h, w]
    (delta, raw density), near / far [b, v] -> two [b, v, h w] maps (tsplat_depth_tail_fwd; see
    oracle.depth_tail)."""
    lib = _lib.load()
    b, v = near.shape
    hw = fullres.shape[-2] * fullres.shape[-1]
    fr, hd, nr, fa = _f32(fullres), _f32(head), _f32(near), _f32(far)
    depth = torch.empty((b, v, hw), dtype=torch.float32, device=fullres.device)
    dens = torch.empty_like(depth)
    _lib.check(lib.tsplat_depth_tail_fwd(_lib.ptr(fr), _lib.ptr(hd), _lib.ptr(nr), _lib.ptr(fa), _lib.ptr(depth),
                                         _lib.ptr(dens), b, v, hw, _lib.stream_ptr(fullres.device)),
               "tsplat_depth_tail_fwd")
    return depth, dens


# DINOv2's attention in split-bf16 precision inside dense_precision("bf16x3") (tsplat_mha_x3_fwd) for
# up to _MHA_X3_ROWS tokens per call: same-box C2 (2 x 325 tokens) 446.9 / 447.8 vs 445.6 / 445.5
# views/s with the exact-fp32 kernel, but C3 (16 x 325) 900.1 / 899.8 vs 903.4 / 902.1 -- there the
# split pass over the 48 MB qkv costs what the cheaper products save (profiles/r5/late/ab_mha_x3.txt).
# TSPLAT_MHA_X3=0 keeps the exact-fp32 kernel in that mode (A/B knob)
_MHA_X3 = os.environ.get("TSPLAT_MHA_X3", "1") == "1"
_MHA_X3_ROWS = 2048


_MHA_PRESPLIT = os.environ.get("TSPLAT_MHA_PRESPLIT", "1") == "1"  # A/B knob (DINOv2 qkv -> split output)


def mha_x3_ok(rows: int) -> bool:
    """True when DINOv2's qkv GEMM hands the bf16x3 attention pre-split operands (mha's default
    precision in the current mode is bf16x3 for `rows` = B * N tokens)."""
    return _MHA_PRESPLIT and _MHA_X3 and _DENSE == "bf16x3" and rows <= _MHA_X3_ROWS


def mha_presplit(qkv_split, heads: int, scale: float):
    """mha in bf16x3 on q / k / v already split: qkv_split [2, B, N, 3 * heads * 64] bf16 (hi, lo;
    gemm_x3(..., act="split")) -> [B, N, heads * 64] fp32 (tsplat_mha_x3_presplit_fwd)."""
    lib = _lib.load()
    _, b, n, c3 = qkv_split.shape
    d = c3 // (3 * heads)
    x = qkv_split.contiguous()
    out = torch.empty((b, n, heads * d), dtype=torch.float32, device=x.device)
    _lib.check(lib.tsplat_mha_x3_presplit_fwd(_lib.ptr(x[0]), _lib.ptr(x[1]), _lib.ptr(out), b, n, heads, d, float(scale),
                                              _lib.stream_ptr(x.device)), "tsplat_mha_x3_presplit_fwd")
    return out


def mha(qkv, heads: int, scale: float, bias=None, precision: str | None = None):
    """Multi-head self-attention from the qkv projection output [B, N, 3 * heads * 64] ->
    [B, N, heads * 64] (tsplat_mha_f32_fwd; no permute copies). bias: the projection's bias when
    qkv was computed without it (tsplat_mha_bias_f32_fwd folds it in). precision "bf16x3" (default:
    the dense mode's, see _MHA_X3) runs tsplat_mha_x3_fwd."""
    lib = _lib.load()
    b, n, c3 = qkv.shape
    d = c3 // (3 * heads)
    x = _f32(qkv)
    out = torch.empty((b, n, heads * d), dtype=torch.float32, device=qkv.device)
    if precision is None:
        precision = "bf16x3" if _MHA_X3 and _DENSE == "bf16x3" and b * n <= _MHA_X3_ROWS else "fp32"
    if precision == "bf16x3":
        ws = torch.empty(int(lib.tsplat_mha_x3_workspace_bytes(b, n, heads, d)), dtype=torch.uint8, device=x.device)
        _lib.check(lib.tsplat_mha_x3_fwd(_lib.ptr(x), _lib.ptr(_f32(bias)) if bias is not None else None,
                                         _lib.ptr(out), _lib.ptr(ws), b, n, heads, d, float(scale),
                                         _lib.stream_ptr(qkv.device)), "tsplat_mha_x3_fwd")
        return out
    if bias is not None:
        _lib.check(lib.tsplat_mha_bias_f32_fwd(_lib.ptr(x), _lib.ptr(_f32(bias)), _lib.ptr(out), b, n, heads, d,
                                               float(scale), _lib.stream_ptr(qkv.device)), "tsplat_mha_bias_f32_fwd")
        return out
    _lib.check(lib.tsplat_mha_f32_fwd(_lib.ptr(x), _lib.ptr(out), b, n, heads, d, float(scale),
                                      _lib.stream_ptr(qkv.device)), "tsplat_mha_f32_fwd")
    return out


# packed weights per weight tensor: id -> (weakref, version, packed); a hit needs the same live
# tensor (never a new tensor at a recycled address or id) at an unchanged version
_CONV_PACKED: dict = {}
# Which convolutions go to tsplat_conv2d_f32_fwd: "auto" (the latency-bound ones, see
# conv2d_direct_ok), "off" (always MIOpen), "all" (every shape the kernel takes; tests / A/B)
_CONV_MODE = os.environ.get("TSPLAT_CONV", "auto")
_CONV_KSPLIT = int(os.environ.get("TSPLAT_CONV_KSPLIT", "0"))  # tuning override (tools/bench_conv.py)
_CONV_MAX_FLOP = 1.5e9  # above this MIOpen's kernels are as fast or faster (tools/bench_conv.py)
_SMALL_MAP_DIRECT = os.environ.get("TSPLAT_CONV_SMALLMAP", "1") == "1"
# 1x1 launch shape: grid cap in waves and minimum ci pairs per wave. Same-box A/B (round-2 session script ab_conv1.sh, pruned in round 5):
# 16384 / 8 reads 338.98 / 338.99 views/s vs 337.91 / 337.58 for the 3x3 rule (4096 / 16); 8192 / 16
# and 16384 / 4 sit in between
_CONV1_WAVES = int(os.environ.get("TSPLAT_CONV1_WAVES", "16384"))
_CONV1_PAIRS = int(os.environ.get("TSPLAT_CONV1_PAIRS", "8"))
# the same for 3x3 (round-2 session script ab_conv3.sh, pruned in round 5, same box: 8192 / 2 reads 340.3 / 339.7 views/s vs 339.3 /
# 339.2 at 4096 / 2; 16384 / 1 and 8192 / 1 in between)
_CONV3_WAVES = int(os.environ.get("TSPLAT_CONV3_WAVES", "8192"))
_CONV3_PAIRS = int(os.environ.get("TSPLAT_CONV3_PAIRS", "2"))
# Split of each tile's ci pairs over workgroups (tsplat_conv2d_f32_zsplit_fwd) for few-tile maps:
# doubled while the grid stays within one round of 16-wave workgroups (one per CU) and every wave
# keeps more than _ZSPLIT_MIN pairs (3x3; 1x1: 4x that). A 32 x 32 tile's workgroup loads the
# weights of its 32 output channels over the whole reduction, so on few-tile maps the per-CU ingest
# of those weights, not the MFMAs, sets the time: splitting the reduction over more CUs divides it.
# TSPLAT_CONV_ZSPLIT=0 turns it off, =N caps it at N.
_ZSPLIT = int(os.environ.get("TSPLAT_CONV_ZSPLIT", "-1"))
_ZSPLIT_WGS = int(os.environ.get("TSPLAT_CONV_ZSPLIT_WGS", "256"))
_ZSPLIT_MIN = int(os.environ.get("TSPLAT_CONV_ZSPLIT_MIN", "1"))  # 4 / 2 / 1: C2 413.4 / 415.8 / 417.3 (profiles/r5/ab_zsplit.txt)
# arrival counters of the zsplit launches: one zeroed slab per device, handed out in rotating ranges
# (each launch leaves its range at zero again), so launches in flight on concurrent streams never share
# a counter while the slab holds more tiles than the launches of one step
_ZSPLIT_CNT: dict = {}
_ZSPLIT_SLAB = 1 << 20


def _zsplit_counters(device, tiles: int):
    """A range of `tiles` zeroed arrival counters for one zsplit launch (its last arrivers reset them
    to 0, so a range is clean again once its launch has finished). Ranges rotate through one slab per
    device, in call order: two launches share counters only if 2^20 tiles of other launches were
    handed out between them, i.e. hundreds of steps apart -- never two launches of one step, which
    are the only ones that can run concurrently (the branches' streams join within the step; graph
    replays are ordered on one stream). One slab per stream instead would have to be allocated inside
    a capture (the capture stream is new), i.e. from the graph's private pool."""
    if tiles > _ZSPLIT_SLAB // 16:
        raise ValueError(f"zsplit launch of {tiles} tiles exceeds the counter slab's per-launch share")
    slab = _ZSPLIT_CNT.get(device)
    if slab is None:
        slab = [torch.zeros(_ZSPLIT_SLAB, dtype=torch.int32, device=device), 0]
        _ZSPLIT_CNT[device] = slab
    if slab[1] + tiles > _ZSPLIT_SLAB:
        slab[1] = 0
    view = slab[0][slab[1]:slab[1] + tiles]
    slab[1] += tiles
    return view


def conv_zsplit(tiles: int, pairs: int, ksplit: int, k: int) -> int:
    """Workgroups per output tile for tsplat_conv2d_f32_zsplit_fwd (1 = no split)."""
    if _ZSPLIT == 0:
        return 1
    per_batch = _ZSPLIT_MIN if k == 3 else 4 * _ZSPLIT_MIN
    z = 1
    while (z < 64 and tiles * 2 * z <= _ZSPLIT_WGS and -(-pairs // (ksplit * z)) > per_batch
           and (_ZSPLIT < 0 or 2 * z <= _ZSPLIT)):
        z *= 2
    return z


def conv_pack_weight(weight):
    """[cout, cin, k, k] -> [ceil(cout / 32), k * k, cin / 2, 2, 32] (zero-padded couts), cached per
    weight tensor version: the A-operand order of tsplat_conv2d_f32_fwd."""
    hit = _CONV_PACKED.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    co, ci, k = weight.shape[:3]  # a Conv1d weight [cout, cin, 1] packs as the 1x1 it is
    cot = (co + 31) // 32
    w = torch.zeros((cot * 32, ci, k * k), dtype=torch.float32, device=weight.device)
    w[:co] = weight.detach().float().reshape(co, ci, k * k)
    packed = w.reshape(cot, 32, ci // 2, 2, k * k).permute(0, 4, 2, 3, 1).contiguous()
    if len(_CONV_PACKED) > 512:
        for k in [k for k, v in _CONV_PACKED.items() if v[0]() is None]:
            del _CONV_PACKED[k]
    _CONV_PACKED[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


def conv2d_direct_ok(x, weight, stride: int = 1, padding=None, c2: int = 0, upsample: bool = False,
                     force: bool = False) -> bool:
    """True when tsplat_conv2d_f32_fwd takes this convolution and (mode "auto") it is a
    latency-bound one where the direct kernel beats MIOpen (force: whenever it takes it)."""
    if _CONV_MODE == "off" or not x.is_cuda or torch.is_autocast_enabled("cuda"):
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() != 4:
        return False
    if weight.dim() == 3:  # Conv1d, kernel 1, on x viewed as [n, c, t, 1]
        if weight.shape[-1] != 1:
            return False
        weight = weight.unsqueeze(-1)
    co, ci, k, k2 = weight.shape
    if k != k2 or k not in (1, 3) or stride not in (1, 2) or (upsample and stride != 1):
        return False
    pad = padding if padding is not None else k // 2
    if isinstance(pad, (tuple, list)):
        if len(set(pad)) != 1:
            return False
        pad = pad[0]
    c1 = x.shape[1]
    if pad != k // 2 or ci != c1 + c2 or c1 % 2 or c2 % 2:
        return False
    if _CONV_MODE == "all" or force:
        return True
    h, w = x.shape[2] * (2 if upsample else 1), x.shape[3] * (2 if upsample else 1)
    npx = x.shape[0] * (h // stride) * (w // stride)
    flop = 2.0 * npx * co * ci * k * k
    # (since the batch loads are scheduled ahead of the MFMAs, the few-tile / long-reduction 3x3s
    # -- 2 x 256 -> 128 at 16^2 -- also beat MIOpen: 23.5 vs 25.7 us, bench_conv.py)
    if _SMALL_MAP_DIRECT and npx <= 512:
        return True  # tiny maps with long reductions (the DPT's 768 -> 768 stride-2 at 18^2, 1.7 GFLOP)
    return flop <= _CONV_MAX_FLOP


# the direct convolutions in the bf16x3 dense mode on split-bf16 MFMA (tsplat_conv2d_bf16x3_fwd) instead of
# exact fp32; TSPLAT_CONV_X3=0 keeps them exact (A/B knob)
_CONV_X3 = os.environ.get("TSPLAT_CONV_X3", "1") == "1"
_CONV_X3_PACKED: dict = {}


def conv_pack_weight_x3(weight):
    """[cout, cin, k, k] -> hi / lo bf16 fragments [ceil(cout / 32)][k * k][ceil(cin / 16)][hi, lo][64 lanes]
    [8] (lane l: cout 32 cot + (l & 31), cin 16 g + 8 (l >> 5) + j; zero-padded), cached per weight
    tensor version: the A operand of tsplat_conv2d_bf16x3_fwd."""
    hit = _CONV_X3_PACKED.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    co, ci = weight.shape[:2]
    k = weight.shape[2] if weight.dim() == 4 else 1
    cot, ng = (co + 31) // 32, (ci + 15) // 16
    w = torch.zeros((cot * 32, ng * 16, k * k), dtype=torch.float32, device=weight.device)
    w[:co, :ci] = weight.detach().float().reshape(co, ci, k * k)
    a = w.reshape(cot, 32, ng, 2, 8, k * k).permute(0, 5, 2, 3, 1, 4)  # [cot, tap, g, h, m, j]
    hi = a.to(torch.bfloat16)
    lo = (a - hi.float()).to(torch.bfloat16)
    packed = torch.stack((hi, lo), dim=3).contiguous()  # [cot, tap, g, hl, h, m, j]
    if len(_CONV_X3_PACKED) > 512:
        for key in [key for key, v in _CONV_X3_PACKED.items() if v[0]() is None]:
            del _CONV_X3_PACKED[key]
    _CONV_X3_PACKED[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


def conv_x3_wins(npx: int, ci: int, co: int, k: int) -> bool:
    """Where the split-bf16 direct kernel beats the exact-fp32 one (graph-timed census of the C2 step,
    profiles/r5/conv_x3/): every 1x1 (one 16-channel unit carries 16 channels' products: 0.8-12 us
    faster per shape), and the 3x3s with >= 0.5 GFLOP over >= 64 input channels (the 768 -> 768
    stride-2 level 53.6 vs 73.6 us). The few-channel / small-map 3x3s stay exact fp32: 32-channel
    3x3s lost 1-2 us each (18 units of 8 gathered channels over 16 waves)."""
    if k == 1:
        return True
    return ci >= 64 and 2.0 * npx * co * ci * k * k >= 0.5e9


def _conv2d_direct_x3(lib, a, b, c1, c2, weight, bias, n, h, w, co, k, stride, upsample, y):
    hout, wout = y.shape[2], y.shape[3]
    tiles = ((n * hout * wout + 31) // 32) * ((co + 31) // 32)
    units = (c1 + c2 + 15) // 16 * k * k
    # waves per tile: up to 16 while the grid stays <= 8192 waves and every wave has a unit; then
    # workgroups per tile (zsplit) doubled while the grid stays within 256 workgroups and every
    # wave keeps >= 2 units (the alternative, >= 1 unit with 4-unit batches, measured slower:
    # profiles/r5/conv_x3/census_x3b.log)
    ksplit = 16
    while ksplit > 1 and (tiles * ksplit > _CONV3_WAVES or units < ksplit):
        ksplit //= 2
    z = 1
    if _ZSPLIT != 0:
        while (z < 64 and tiles * 2 * z <= _ZSPLIT_WGS and units >= 2 * ksplit * 2 * z
               and (_ZSPLIT < 0 or 2 * z <= _ZSPLIT)):
            z *= 2
    part = cnt = None
    if z > 1:
        part = torch.empty(tiles * z * 1024, dtype=torch.float32, device=y.device)
        cnt = _zsplit_counters(y.device, tiles)
    pb = _f32(bias) if bias is not None else None
    rc = lib.tsplat_conv2d_bf16x3_fwd(_lib.ptr(a), c1, _lib.ptr(b), c2, _lib.ptr(conv_pack_weight_x3(weight)),
                                      _lib.ptr(pb), _lib.ptr(y), n, h, w, co, k, stride, int(upsample), ksplit, z,
                                      _lib.ptr(part), _lib.ptr(cnt), _lib.stream_ptr(y.device))
    _lib.check(rc, "tsplat_conv2d_bf16x3_fwd")
    return y


def conv2d_direct(x1, weight, bias=None, stride: int = 1, x2=None, upsample: bool = False):
    """conv2d(cat([x1, x2], 1) (nearest-upsampled 2x if upsample), weight, bias, stride,
    padding = k // 2) in one MFMA launch, NCHW fp32: exact fp32 (tsplat_conv2d_f32_zsplit_fwd), or
    split-bf16 in the bf16x3 dense mode (tsplat_conv2d_bf16x3_fwd)."""
    lib = _lib.load()
    n, c1, h, w = x1.shape
    a = _f32(x1)
    b = _f32(x2) if x2 is not None else None
    c2 = b.shape[1] if b is not None else 0
    if b is not None and (b.shape[0] != n or b.shape[2:] != x1.shape[2:]):
        raise ValueError(f"x2 {tuple(b.shape)} does not match x1 {tuple(x1.shape)}")
    co, ci, k = weight.shape[:3]
    if ci != c1 + c2:
        raise ValueError(f"weight {tuple(weight.shape)} does not match {c1} + {c2} input channels")
    hv, wv = (2 * h, 2 * w) if upsample else (h, w)
    hout, wout = (hv + 2 * (k // 2) - k) // stride + 1, (wv + 2 * (k // 2) - k) // stride + 1
    y = torch.empty((n, co, hout, wout), dtype=torch.float32, device=x1.device)
    if _CONV_X3 and split_mode() and conv_x3_wins(n * hout * wout, c1 + c2, co, k):
        return _conv2d_direct_x3(lib, a, b, c1, c2, weight, bias, n, h, w, co, k, stride, upsample, y)
    # waves per 32 x 32 tile: the ci pairs split over up to 16 waves (>= 2 pairs of a 3x3 each while
    # the grid stays <= 8192 waves; >= 8 pairs of a 1x1 each up to 16384 waves: its waves are short,
    # one or two batches of loads, so more of them in flight hide more of the latency)
    tiles = ((n * hout * wout + 31) // 32) * ((co + 31) // 32)
    pairs = ci // 2
    ksplit = 16
    cap, min_pairs = (_CONV3_WAVES, _CONV3_PAIRS) if k == 3 else (_CONV1_WAVES, _CONV1_PAIRS)
    while ksplit > 1 and (tiles * ksplit > cap or pairs < min_pairs * ksplit):
        ksplit //= 2
    ksplit = _CONV_KSPLIT or ksplit
    zsplit = conv_zsplit(tiles, pairs, ksplit, k) if ksplit == 16 else 1
    pb = _f32(bias) if bias is not None else None
    part = cnt = None
    if zsplit > 1:
        part = torch.empty(tiles * zsplit * 1024, dtype=torch.float32, device=x1.device)
        cnt = _zsplit_counters(x1.device, tiles)
    rc = lib.tsplat_conv2d_f32_zsplit_fwd(_lib.ptr(a), c1, _lib.ptr(b), c2, _lib.ptr(conv_pack_weight(weight)),
                                          _lib.ptr(pb), _lib.ptr(y), n, h, w, co, k, stride, int(upsample), ksplit,
                                          zsplit, _lib.ptr(part), _lib.ptr(cnt), _lib.stream_ptr(x1.device))
    _lib.check(rc, "tsplat_conv2d_f32_zsplit_fwd")
    return y


# Winograd-transformed weights per weight tensor (same caching rule as _CONV_PACKED)
_WINO_PACKED: dict = {}
# Which 3x3 convolutions go to tsplat_conv3x3_wino_f32_fwd: "auto" (the shapes where it beats
# MIOpen, see conv3x3_wino_ok), "off", "all" (every 3x3 / stride 1 / pad 1 fp32 conv; tests / A/B),
# "big" (auto with the direct kernel's FLOP floor also where MIOpen is the alternative; A/B only:
# same box 322.1 / 322.9 vs auto 323.4 / 323.7 views/s)
_WINO_MODE = os.environ.get("TSPLAT_WINO", "auto")
_WINO_ACT = {"none": 0, "relu": 1, "gelu": 2}


def wino_pack_weight(weight):
    """[cout, cin, 3, 3] -> the transformed filters G g G^T in the A-operand order of
    tsplat_conv3x3_wino_f32_fwd, cached per weight tensor version."""
    hit = _WINO_PACKED.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    lib = _lib.load()
    co, ci = weight.shape[:2]
    packed = torch.empty(int(lib.tsplat_wino_weight_floats(co, ci)), dtype=torch.float32, device=weight.device)
    w = weight.detach().float().contiguous()
    _lib.check(lib.tsplat_wino_weight_f32(_lib.ptr(w), _lib.ptr(packed), co, ci, _lib.stream_ptr(weight.device)),
               "tsplat_wino_weight_f32")
    if len(_WINO_PACKED) > 512:
        for k in [k for k, v in _WINO_PACKED.items() if v[0]() is None]:
            del _WINO_PACKED[k]
    _WINO_PACKED[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


WINO_MAX_CI_PAD = 1024  # winoconv.hip kMaxCiPad: input channels (padded to 16) of one launch


def conv3x3_wino_ok(x, weight, stride=1, padding=1, dilation=1, groups=1, extra=(), vs_miopen=False,
                    force=False) -> bool:
    """True when tsplat_conv3x3_wino_f32_fwd takes conv2d(x, weight) on the NCHW map x and (mode
    "auto") it is one of the 3x3s where it beats MIOpen's kernels (tools/bench_wino.py): above the
    direct kernel's FLOP range (unless `vs_miopen`: the caller's alternative is MIOpen, which the
    Winograd kernel also beats below that range, e.g. 96 -> 96 at 64^2: 20.8 vs 27.1 us), and not
    the few-tile / long-reduction shapes (256 input channels at 32^2: 64 workgroups of 32 serial
    chunks) where MIOpen stays faster."""
    if _WINO_MODE == "off" or not x.is_cuda or torch.is_autocast_enabled("cuda") or len(extra) > 5:
        return False
    for t in (x, *extra):
        if (t.dtype != torch.float32 or t.dim() != 4 or not t.is_contiguous() or t.device != x.device
                or t.shape[0] != x.shape[0] or t.shape[2:] != x.shape[2:]):
            return False
    if weight.dtype != torch.float32 or weight.dim() != 4:
        return False
    as_int = lambda v: v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else -1)
    if tuple(weight.shape[2:]) != (3, 3) or as_int(stride) != 1 or as_int(padding) != 1:
        return False
    ci = sum(t.shape[1] for t in (x, *extra))
    if as_int(dilation) != 1 or groups != 1 or weight.shape[1] != ci:
        return False
    if (ci + 15) // 16 * 16 > WINO_MAX_CI_PAD:  # the launch's LDS plane table (winoconv.hip kMaxCiPad)
        return False
    if _WINO_MODE == "all" or force:
        return True
    n, _, h, w = x.shape
    co = weight.shape[0]
    groups_ = n * ((h + 1) // 2 * ((w + 1) // 2) + 31) // 32 * ((co + 31) // 32)  # ~ workgroups
    vs_miopen = vs_miopen and _WINO_MODE != "big"  # "big": the FLOP floor everywhere (A/B knob)
    # (a head with a handful of output channels on a large map -- 64 -> 2 at 256^2 -- still beats
    # MIOpen's 53 us with one mostly idle 32-channel output block: the transform dominates there)
    return (ci >= 16 and (co >= 16 or (vs_miopen and n * h * w >= 65536))
            and (vs_miopen or 2.0 * n * h * w * co * ci * 9 > _CONV_MAX_FLOP)
            and (ci <= 192 or groups_ >= 256))


_ENC_DIRECT = os.environ.get("TSPLAT_ENC_DIRECT", "1") != "0"  # A/B knob for conv2d_forward's direct route


def conv2d_forward(mod, x):
    """nn.Conv2d.forward (installed on the encoder's Conv2d modules by install_conv2d_dispatch):
    the 3x3s that conv3x3_wino_ok admits on the Winograd kernel, the latency-bound 1x1 / 3x3
    (stride 1 or 2) ones that conv2d_direct_ok admits on the direct kernel (bias in the epilogue
    instead of MIOpen's separate bias launch), the rest through MIOpen."""
    if mod.padding_mode == "zeros" and mod.groups == 1 and tuple(mod.dilation) == (1, 1):
        if conv_bf16_ok(x, mod.weight, mod.stride, mod.padding, mod.dilation, mod.groups):
            return conv_bf16(x, mod.weight, mod.bias)
        if conv3x3_wino_ok(x, mod.weight, mod.stride, mod.padding, mod.dilation, mod.groups, vs_miopen=True):
            return conv3x3_wino(x, mod.weight, mod.bias)
        st = mod.stride[0] if mod.stride[0] == mod.stride[1] else 0
        if (_ENC_DIRECT and st and x.is_contiguous() and x.dtype == torch.float32
                and conv2d_direct_ok(x, mod.weight, st, mod.padding)):
            return conv2d_direct(x, mod.weight, mod.bias, st)
        y = _conv2d_x3_libfree(x, mod.weight, mod.bias, mod.stride, mod.padding)
        if y is not None:
            return y
        k = mod.kernel_size
        if (_LIBFREE and st and k[0] == k[1] and k[0] > 3 and mod.padding[0] == mod.padding[1] and x.is_cuda
                and x.dtype == torch.float32 and mod.weight.dtype == torch.float32
                and not torch.is_autocast_enabled("cuda")):
            return conv_unfold_gemm(x, mod.weight, mod.bias, st, mod.padding[0])
    return mod._conv_forward(x, mod.weight, mod.bias)


# Convolutions the encoder used to leave on MIOpen (round 5): the UniMatch CNN's 7x7 stride-2 stem
# and the DPT's transposed convolutions (kernel = stride). MIOpen picks their algorithms by timing
# (cudnn.benchmark), so their bits could differ from process to process; these forms are exact fp32
# and fixed. TSPLAT_CONV_LIBFREE=0 keeps them on MIOpen (A/B knob).
_LIBFREE = os.environ.get("TSPLAT_CONV_LIBFREE", "1") == "1"
# bf16x3 mode: every remaining Conv2d on the split-bf16 Winograd / direct kernels (TSPLAT_CONV_LIBFREE_X3=0:
# the shapes above the latency-bound range stay on MIOpen, the A/B knob)
_LIBFREE_X3 = os.environ.get("TSPLAT_CONV_LIBFREE_X3", "1") == "1"
_DERIVED: dict = {}


def _derived(weight, tag, make):
    """A tensor derived from `weight` (cached per weight tensor and version, like _CONV_PACKED)."""
    key = (id(weight), tag)
    hit = _DERIVED.get(key)
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    val = make(weight.detach())
    if len(_DERIVED) > 256:
        for k in [k for k, v in _DERIVED.items() if v[0]() is None]:
            del _DERIVED[k]
    _DERIVED[key] = (weakref.ref(weight), weight._version, val)
    return val


def conv_unfold_gemm(x, weight, bias, stride: int, padding: int):
    """conv2d(x, weight, bias, stride, padding) as im2col (F.unfold) + one exact-fp32 GEMM: the
    7x7 stride-2 stem on 3 channels (reference backbone/unimatch CNN conv1), which the direct and
    Winograd kernels do not take."""
    n, ci, h, w = x.shape
    co, _, kh, kw = weight.shape
    ho, wo = (h + 2 * padding - kh) // stride + 1, (w + 2 * padding - kw) // stride + 1
    cols = torch.nn.functional.unfold(x, (kh, kw), padding=padding, stride=stride)  # [n, ci kh kw, L]
    # one GEMM per image straight into its [co, L] slab, bias in the GEMM's C term (a broadcast
    # matmul over the batch transposed cols into a [n L, ci kh kw] copy first, and the bias add
    # was another pass)
    wm = weight.reshape(co, -1)
    y = torch.empty((n, co, ho * wo), dtype=torch.float32, device=x.device)
    with torch.autocast("cuda", enabled=False):
        for i in range(n):
            if bias is not None:
                torch.addmm(bias.view(co, 1), wm, cols[i], out=y[i])
            else:
                torch.mm(wm, cols[i], out=y[i])
    return y.view(n, co, ho, wo)


def conv_transpose_direct(x, weight, bias, s: int):
    """conv_transpose2d(x, weight [ci, co, s, s], bias, stride s) -- the DPT's resize_layers
    (kernel = stride, no overlap, reference dpt.py:105-118): a 1x1 convolution to co * s^2 channels
    on the direct exact-fp32 kernel (bias in its epilogue) + pixel_shuffle (a copy)."""
    ci, co = weight.shape[:2]
    w1 = _derived(weight, "convT", lambda t: t.permute(1, 2, 3, 0).reshape(co * s * s, ci, 1, 1).contiguous())
    b1 = _derived(bias, "convT_b", lambda t: t.repeat_interleave(s * s).contiguous()) if bias is not None else None
    return torch.nn.functional.pixel_shuffle(conv2d_direct(x, w1, b1, 1), s)


def conv_transpose_forward(mod, x):
    """nn.ConvTranspose2d.forward (installed by install_conv2d_dispatch): kernel = stride, no padding
    -> conv_transpose_direct; anything else through MIOpen."""
    k, st = mod.kernel_size, mod.stride
    if (_LIBFREE and k[0] == k[1] == st[0] == st[1] and tuple(mod.padding) == (0, 0) and mod.groups == 1
            and tuple(mod.output_padding) == (0, 0) and tuple(mod.dilation) == (1, 1) and x.is_cuda
            and x.dtype == torch.float32 and mod.weight.dtype == torch.float32 and x.shape[1] % 2 == 0
            and not torch.is_autocast_enabled("cuda")):
        return conv_transpose_direct(x.contiguous(), mod.weight, mod.bias, st[0])
    return torch.nn.ConvTranspose2d.forward(mod, x)


def _conv2d_x3_libfree(x, weight, bias, stride, padding):
    """bf16x3 mode, a convolution the shape rules leave to MIOpen (C3's b = 8 levels): the split-bf16
    Winograd for the 3x3 / stride-1 ones up to 256 input channels, the direct kernel for the rest --
    per shape within ~1.4x of MIOpen either way, 1.26 vs 1.28 ms over C3's 18 such calls
    (tools/c3_libconv.py, profiles/r6/c3_libconv.log), and no library convolution left. None when
    the shape is not one of those (or TSPLAT_CONV_LIBFREE_X3=0, or another mode)."""
    if not (_LIBFREE_X3 and split_mode() and x.is_cuda and x.dim() == 4 and x.is_contiguous()
            and x.dtype == torch.float32 and weight.dim() == 4):
        return None
    st = stride if isinstance(stride, int) else (stride[0] if stride[0] == stride[1] else 0)
    if not st:
        return None
    if weight.shape[1] <= 256 and conv3x3_wino_ok(x, weight, stride, padding, force=True):
        return conv3x3_wino(x, weight, bias)
    if conv2d_direct_ok(x, weight, st, padding, force=True):
        return conv2d_direct(x, weight, bias, st)
    return None


def conv2d_fallback(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """F.conv2d for the model code's last-resort branches: in the bf16x3 mode through
    _conv2d_x3_libfree first, so no convolution of that mode reaches MIOpen."""
    if groups == 1 and (dilation == 1 or tuple(dilation) == (1, 1)):
        y = _conv2d_x3_libfree(x, weight, bias, stride, padding)
        if y is not None:
            return y
    return torch.nn.functional.conv2d(x, weight, bias, stride, padding, dilation, groups)


def install_conv2d_dispatch(module) -> int:
    """Route every nn.Conv2d under `module` through conv2d_forward (same parameters, same state
    dict); returns the number of modules routed."""
    import functools

    n = 0
    for m in module.modules():
        if type(m) is torch.nn.Conv2d:
            m.forward = functools.partial(conv2d_forward, m)
            n += 1
        elif type(m) is torch.nn.ConvTranspose2d:
            m.forward = functools.partial(conv_transpose_forward, m)
            n += 1
    return n


# Dense-layer precision of the fp32 path (set by the encoder around its dense regions,
# EncoderTransCfg.dense_dtype): "fp32" = exact fp32 MFMA / library SGEMM; "bf16x3" = split-bf16
# products (x = hi + lo, hi*hi + hi*lo + lo*hi on bf16 MFMA, fp32 accumulation: <= 3 * 2^-18
# relative per product, the stand-in for the reference's TF32, src/main.py:15).
_DENSE = "fp32"
_DENSE_MODES = ("fp32", "bf16x3")


# bf16x3 mode's OTHER library fp32 GEMMs (the ones linear_xf32 below does not admit): with
# TSPLAT_XF32=1 the whole dense_precision("bf16x3") block runs with torch's allow_tf32, which on
# gfx950 selects hipBLASLt's emulated-xf32 kernels (fp32 in / out, bf16 MFMA; tools/bench_xf32.py
# measures their error next to the split kernels'). Off by default; independently of it, the linears
# linear_xf32_ok admits (on by default, TSPLAT_LINX) always run under allow_tf32 -- see linear_xf32.
_XF32 = os.environ.get("TSPLAT_XF32", "0") == "1"


class dense_precision:
    """Context manager: the dense-layer precision mode inside the block (see _DENSE)."""

    def __init__(self, mode: str):
        if mode not in _DENSE_MODES:
            raise ValueError(f"dense precision {mode!r} not in {_DENSE_MODES}")
        self.mode, self.prev, self.prev_tf32 = mode, None, None

    def __enter__(self):
        global _DENSE
        self.prev, _DENSE = _DENSE, self.mode
        self.prev_tf32 = torch.backends.cuda.matmul.allow_tf32
        torch.backends.cuda.matmul.allow_tf32 = _XF32 and self.mode == "bf16x3"
        return self

    def __exit__(self, *exc):
        global _DENSE
        _DENSE = self.prev
        torch.backends.cuda.matmul.allow_tf32 = self.prev_tf32
        return False


def split_mode() -> bool:
    """True inside dense_precision("bf16x3")."""
    return _DENSE == "bf16x3"


# Window-attention precision of the fp32 transformer path: "fp32" (exact fp32 MFMA), "bf16x3"
# (split-bf16 products on bf16 MFMA, fp32 softmax: the bf16x3 dense mode's attention, >= the
# reference's TF32; tsplat_win_attn_x3_*, where the launch splits the keys -- else exact fp32) or
# "bf16" (q / k / v rounded to bf16, bf16 MFMA with fp32 softmax and accumulation: config C3's "bf16
# attention" beside fp32-class dense layers). Under bf16 autocast the attention is bf16 regardless.
_ATTN = "fp32"
ATTN_MODES = ("fp32", "bf16x3", "bf16")


def auto_attention(dense_dtype: str) -> str:
    """The attention precision "auto" means beside `dense_dtype` (TSPLAT_ATTN_X3=0: exact fp32
    attention in the bf16x3 dense mode, the A/B knob)."""
    if dense_dtype == "bf16":
        return "bf16"
    return "bf16x3" if dense_dtype == "bf16x3" and _ATTN_X3 else "fp32"


class attention_precision:
    """Context manager: the window-attention precision inside the block (see _ATTN)."""

    def __init__(self, mode: str):
        if mode not in ATTN_MODES:
            raise ValueError(f"attention precision {mode!r}")
        self.mode, self.prev = mode, None

    def __enter__(self):
        global _ATTN
        self.prev, _ATTN = _ATTN, self.mode
        return self

    def __exit__(self, *exc):
        global _ATTN
        _ATTN = self.prev
        return False


_SPLIT_W: dict = {}


def split_bf16x3(x: torch.Tensor, weight_order: bool = False) -> torch.Tensor:
    """[..., k] fp32 -> [..., 3k] bf16: [hi | hi | lo] (activations) or [hi | lo | hi] (weights_order),
    hi = bf16(x), lo = bf16(x - hi) (tsplat_split_bf16x3)."""
    lib = _lib.load()
    xf = _f32(x)
    k = xf.shape[-1]
    out = torch.empty((*xf.shape[:-1], 3 * k), dtype=torch.bfloat16, device=xf.device)
    _lib.check(lib.tsplat_split_bf16x3(_lib.ptr(xf), _lib.ptr(out), xf.numel() // k, k, int(weight_order),
                                       _lib.stream_ptr(xf.device)), "tsplat_split_bf16x3")
    return out


def _split_weight(weight):
    """[n, k] -> [n, 3k] bf16 [hi | lo | hi], cached per weight tensor version."""
    hit = _SPLIT_W.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    packed = split_bf16x3(weight.detach(), weight_order=True)
    if len(_SPLIT_W) > 512:
        for k in [k for k, v in _SPLIT_W.items() if v[0]() is None]:
            del _SPLIT_W[k]
    _SPLIT_W[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


def linear_bf16x3(x, weight, bias=None, act: str = "none", cache: bool = True):
    """act(F.linear(x, weight, bias)) in split-bf16 precision (act "none" or "gelu", exact erf) as ONE
    hipBLASLt bf16 GEMM with K' = 3K on [x_hi | x_hi | x_lo] and [W_hi | W_lo | W_hi] (fp32
    accumulation and output); W packed once per version (cache=False: for this call only, for a
    weight that is an activation). Round 4's hand-written split GEMM for DINOv2's M = 650 linears
    (csrc/gemm3.hip) measured slower than the library in the step (C2 381 vs 394 views/s,
    profiles/r4/g12/: at M = 650 bf16x3 cuts the MFMA cycles but not the fp32-sized operand bytes)
    and was removed from the library in round 5."""
    k, n = x.shape[-1], weight.shape[0]
    w3 = _split_weight(weight) if cache else split_bf16x3(weight, weight_order=True)
    x3 = split_bf16x3(x).reshape(-1, 3 * k)
    with torch.autocast("cuda", enabled=False):
        if bias is not None:
            y = torch.addmm(_f32(bias), x3, w3.t(), out_dtype=torch.float32)
        else:
            y = torch.mm(x3, w3.t(), out_dtype=torch.float32)
    y = y.reshape(*x.shape[:-1], n)
    if act == "gelu":
        y = torch.nn.functional.gelu(y)
    return y


# Library fp32 GEMMs in bf16x3 mode: hipBLASLt's emulated-xf32 kernels (fp32 in / out on bf16 MFMA;
# selected by torch's allow_tf32 for a plain matmul, not for addmm with a bias epilogue) measured
# 4.4-5.6e-6 of max |y| against float64 -- the bf16x3 class, TF32-emulated operands 2.0-2.4e-4 -- and
# faster where N >= 1024 or M >= 4096 (tools/bench_xf32.py, profiles/r4/g12/xf32_tf32.log: DINOv2
# qkv 20.7 vs 29.6 us, fc1 25.7 vs 30.5, MVT fc1 22.8 vs 39.2; proj / fc2 at N = 768 slower: they stay
# exact fp32). The bias (+ exact GELU) then runs as one pass (tsplat_bias_act_nhwc_fwd on [rows, N]).
# OFF by default since round 6: with these emulated-xf32 library GEMMs in the step (DINOv2's on the
# current stream beside the backbone branch's library GEMMs on the side stream), hipGraph replays of
# the C2 step were NOT the eager step: 1-3 of 4 replays moved 0.6-4 % of the pixels by up to 4e-2
# (tools/graph_vs_eager.py, profiles/r6/graph_vs_eager.log), with every library GEMM exact fp32 8 of
# 8 replays were bit-identical to eager. TSPLAT_LINX=1 restores the route (A/B only);
# TSPLAT_LINX_SIDE=0 with it keeps it off the side streams (measured: still racing).
_LINX = os.environ.get("TSPLAT_LINX", "0") == "1"
_LINX_SIDE = os.environ.get("TSPLAT_LINX_SIDE", "1") == "1"


def linear_xf32_ok(x, weight) -> bool:
    """True when linear_forward takes linear_xf32 for F.linear(x, weight) in the current mode."""
    if not (_LINX and _DENSE == "bf16x3" and x.is_cuda and x.dtype == torch.float32
            and weight.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")):
        return False
    n, k = weight.shape
    m = x.numel() // max(k, 1)
    if not _LINX_SIDE:
        from . import streams

        if streams._is_side(torch.cuda.current_stream(x.device)):
            return False
    return n % 4 == 0 and ((n >= 1024 and m >= 512) or (m >= 4096 and n >= 512))


def linear_xf32(x, weight, bias=None, act: str = "none"):
    """act(x W^T + bias) with the product on hipBLASLt's emulated-xf32 kernels (see _LINX) and the
    bias / activation in one tsplat_bias_act_nhwc_fwd pass."""
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = True
    try:
        y = torch.matmul(x, weight.t())
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
    if bias is None and act == "none":
        return y
    y = y.contiguous()
    bb = _f32(bias) if bias is not None else None
    lib = _lib.load()
    rc = lib.tsplat_bias_act_nhwc_fwd(_lib.ptr(y), _lib.ptr(bb), None, None, _lib.ptr(y), y.numel() // y.shape[-1],
                                      y.shape[-1], _ACTS[act], _lib.stream_ptr(y.device))
    _lib.check(rc, "tsplat_bias_act_nhwc_fwd")
    return y


# Hand-written split-bf16 GEMM (tsplat_gemm_x3_fwd) for the bf16x3 mode's DINOv2 linears (round 6):
# replaces hipBLASLt's exact-fp32 / emulated-xf32 GEMMs there. TSPLAT_GEMM_X3=0: the library path.
_GEMM_X3 = os.environ.get("TSPLAT_GEMM_X3", "1") == "1"
_GEMM_KSPLIT = int(os.environ.get("TSPLAT_GEMM_KSPLIT", "0"))  # 0: auto
_GEMM_W: dict = {}
GEMM_LOG = None  # list: (m, n, k, ksplit) per launch when set (bench.py's roofline)


def gemm_x3_ok(x, weight) -> bool:
    """True when gemm_x3 takes F.linear(x, weight) in the current mode: bf16x3 dense mode, fp32 on
    the GPU, k and n multiples of 4."""
    if not (_GEMM_X3 and _DENSE == "bf16x3" and x.is_cuda and x.dtype == torch.float32
            and weight.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")):
        return False
    n, k = weight.shape
    return k % 4 == 0 and n % 4 == 0 and x.shape[-1] == k


def _gemm_pack(weight):
    """W [n, k] -> its packed hi / lo MFMA fragments, cached per weight tensor version."""
    hit = _GEMM_W.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    lib = _lib.load()
    n, k = weight.shape
    wf = _f32(weight.detach())
    wp = torch.empty(int(lib.tsplat_gemm_x3_pack_bytes(n, k)), dtype=torch.uint8, device=weight.device)
    _lib.check(lib.tsplat_gemm_x3_pack(_lib.ptr(wf), _lib.ptr(wp), n, k, _lib.stream_ptr(weight.device)),
               "tsplat_gemm_x3_pack")
    if len(_GEMM_W) > 512:
        for key in [key for key, v in _GEMM_W.items() if v[0]() is None]:
            del _GEMM_W[key]
    _GEMM_W[id(weight)] = (weakref.ref(weight), weight._version, wp)
    return wp


def gemm_ksplit(m: int, n: int, k: int) -> int:
    """Split-K factor: the tile grid (64-row x 128-column blocks) filled up to one workgroup per CU
    (256; a 257th workgroup doubles a CU's share: DINOv2 fc2 at 3 splits 17.3 us, at 4 21.5,
    profiles/r6/gemm/), every split at least two 64-deep chunks."""
    if _GEMM_KSPLIT > 0:
        return _GEMM_KSPLIT
    tiles = -(-m // 64) * -(-n // 128)
    nchunk = -(-k // 64)
    s = max(1, min(nchunk // 2, 256 // tiles))
    while s > 1 and (s - 1) * -(-nchunk // s) >= nchunk:
        s -= 1
    return s


def gemm_x3(x, weight, bias=None, act: str = "none", ksplit: int = 1):
    """act(x W^T + bias) on the split-bf16 GEMM (tsplat_gemm_x3_fwd); ksplit > 1 returns the [ksplit,
    *x.shape[:-1], n] partial slabs (bias in slab 0) for residual_ln to sum; ksplit 0: gemm_ksplit's
    choice (1 with an activation)."""
    lib = _lib.load()
    n, k = weight.shape
    xf = _f32(x)
    m = xf.numel() // k
    if ksplit == 0:
        ksplit = 1 if act != "none" else gemm_ksplit(m, n, k)
    if act == "split":  # [2, *x.shape[:-1], n] bf16: hi and lo images (x W^T + bias = hi + lo)
        if ksplit != 1:
            raise ValueError("gemm_x3: the split output needs ksplit 1")
        out = torch.empty((2, *x.shape[:-1], n), dtype=torch.bfloat16, device=x.device)
    else:
        shape = (*x.shape[:-1], n) if ksplit == 1 else (ksplit, *x.shape[:-1], n)
        out = torch.empty(shape, dtype=torch.float32, device=x.device)
    if GEMM_LOG is not None:
        GEMM_LOG.append((m, n, k, ksplit))
    rc = lib.tsplat_gemm_x3_fwd(_lib.ptr(xf), _lib.ptr(_gemm_pack(weight)), _lib.ptr(_f32(bias)) if bias is not None else None,
                                _lib.ptr(out), m, n, k, ksplit, {"none": 0, "gelu": 1, "split": 2}[act],
                                _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_gemm_x3_fwd", "bf16x3")
    return out


def linear_forward(mod, x):
    """nn.Linear.forward (installed by install_linear_dispatch): in dense_precision("bf16x3") the fp32
    linears run on the split-bf16 GEMM (gemm_x3; linear_xf32 instead if its A/B knob admits them, and
    F.linear below 64 rows); everything else is F.linear."""
    import torch.nn.functional as F

    if linear_xf32_ok(x, mod.weight):
        return linear_xf32(x, mod.weight, mod.bias)
    if gemm_x3_ok(x, mod.weight) and x.numel() // x.shape[-1] >= 64:
        return gemm_x3(x, mod.weight, mod.bias)
    return F.linear(x, mod.weight, mod.bias)


def install_linear_dispatch(module) -> int:
    """Route every nn.Linear under `module` through linear_forward (same parameters and state dict)."""
    import functools

    n = 0
    for m in module.modules():
        if type(m) is torch.nn.Linear:
            m.forward = functools.partial(linear_forward, m)
            n += 1
    return n


# bench.py's roofline pass sets a list here: one (Winograd GEMM FLOPs, direct-equivalent FLOPs) pair
# per launch (GEMM FLOPs = 2 * 16 * ci * co * output tiles, the products the 16 MFMA GEMMs compute)
WINO_FLOP_LOG = None


_WINO3_PACKED: dict = {}


def wino_pack_weight_bf16x3(weight):
    """[cout, cin, 3, 3] -> G g G^T split into hi / lo bf16 in the A-operand order of
    tsplat_conv3x3_wino_bf16x3_fwd, cached per weight tensor version."""
    hit = _WINO3_PACKED.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    lib = _lib.load()
    co, ci = weight.shape[:2]
    packed = torch.empty(int(lib.tsplat_wino_weight_bf16x3_bytes(co, ci)), dtype=torch.uint8, device=weight.device)
    w = weight.detach().float().contiguous()
    _lib.check(lib.tsplat_wino_weight_bf16x3(_lib.ptr(w), _lib.ptr(packed), co, ci, _lib.stream_ptr(weight.device)),
               "tsplat_wino_weight_bf16x3")
    if len(_WINO3_PACKED) > 512:
        for k in [k for k, v in _WINO3_PACKED.items() if v[0]() is None]:
            del _WINO3_PACKED[k]
    _WINO3_PACKED[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


# bf16x3 3x3s of few-channel full-resolution maps on the direct kernel tsplat_conv3x3_few_bf16x3_fwd
# instead of the Winograd one (TSPLAT_CONV_FEW=0: Winograd everywhere, the A/B knob): <= 32 outputs from
# <= 64 inputs over >= 2 x 256^2 pixels, where it measured faster (2 x 32 -> 32 at 256^2 20.9 vs 25.3 us,
# 64 -> 32 32.1 vs 35.3, 38 -> 32 26.7 vs 29.6; at 64 outputs or 128^2 maps it only ties:
# profiles/r6/few_sweep.log)
_FEW = os.environ.get("TSPLAT_CONV_FEW", "1") != "0"
FEW_MIN_PX = int(os.environ.get("TSPLAT_CONV_FEW_MIN_PX", str(2 * 256 * 256)))
FEW_MAX_CI = int(os.environ.get("TSPLAT_CONV_FEW_MAX_CI", "64"))
FEW_MAX_CO = int(os.environ.get("TSPLAT_CONV_FEW_MAX_CO", "32"))


def _few_ok(srcs, n: int, h: int, w: int, co: int) -> bool:
    ci = sum(t.shape[1] for t in srcs)
    return (_FEW and co <= FEW_MAX_CO and ci <= FEW_MAX_CI and n * h * w >= FEW_MIN_PX and w % 4 == 0
            and all(t.data_ptr() % 16 == 0 for t in srcs)
            and int(_lib.load().tsplat_conv3x3_few_form(n, ci, h, w, co)) != 0)


def conv3x3_wino(x, weight, bias=None, act: str = "none", extra=(), precision: str | None = None, residual=None,
                 residual2=None, relu_in: bool = False):
    """act(conv2d(cat([x, *extra], 1), weight, bias, stride 1, padding 1)) (+ residual + residual2)
    via Winograd F(2x2, 3x3); the concatenation is read in place; relu_in: ReLU on the input as it
    is loaded. precision "fp32" (tsplat_conv3x3_wino_cat_f32_fwd, exact fp32 MFMA; relu_in /
    residuals as separate launches) or "bf16x3" (tsplat_conv3x3_wino_bf16x3_ex_fwd, split-bf16
    MFMA, all fused); default: the current dense_precision mode."""
    import ctypes

    lib = _lib.load()
    precision = precision or _DENSE
    if precision != "bf16x3" and (relu_in or residual is not None or residual2 is not None):
        y = conv3x3_wino(torch.relu(x) if relu_in else x, weight, bias, act,
                         tuple(torch.relu(t) for t in extra) if relu_in else extra, precision)
        for r in (residual, residual2):
            if r is not None:
                y = y + r
        return y
    srcs = [_f32(t) for t in (x, *extra)]
    n, _, h, w = srcs[0].shape
    co = weight.shape[0]
    if WINO_FLOP_LOG is not None:
        ci = sum(t.shape[1] for t in srcs)
        WINO_FLOP_LOG.append((2.0 * 16 * ci * co * n * ((h + 1) // 2) * ((w + 1) // 2), 2.0 * n * h * w * co * ci * 9))
    y = torch.empty((n, co, h, w), dtype=torch.float32, device=x.device)
    pb = _f32(bias) if bias is not None else None
    ptrs = (ctypes.c_void_p * len(srcs))(*[_lib.ptr(t) for t in srcs])
    chans = (ctypes.c_int32 * len(srcs))(*[t.shape[1] for t in srcs])
    if precision == "bf16x3":
        res = [_f32(r) if r is not None else None for r in (residual, residual2)]
        for r in res:
            if r is not None and tuple(r.shape) != tuple(y.shape):
                raise ValueError(f"residual {tuple(r.shape)} != output {tuple(y.shape)}")
        if _few_ok(srcs, n, h, w, co):
            # few-channel full-resolution maps: the direct split-bf16 kernel (csrc/convfew.hip)
            rc = lib.tsplat_conv3x3_few_bf16x3_fwd(
                ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(chans, ctypes.c_void_p), len(srcs),
                _lib.ptr(conv_pack_weight_x3(weight)), _lib.ptr(pb), _lib.ptr(res[0]), _lib.ptr(res[1]),
                _lib.ptr(y), n, h, w, co, _WINO_ACT[act], int(relu_in), _lib.stream_ptr(x.device))
            _lib.check(rc, "tsplat_conv3x3_few_bf16x3_fwd")
            return y
        rc = lib.tsplat_conv3x3_wino_bf16x3_ex_fwd(
            ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(chans, ctypes.c_void_p), len(srcs),
            _lib.ptr(wino_pack_weight_bf16x3(weight)), _lib.ptr(pb), _lib.ptr(res[0]), _lib.ptr(res[1]), _lib.ptr(y),
            n, h, w, co, _WINO_ACT[act], int(relu_in), _lib.stream_ptr(x.device))
        _lib.check(rc, "tsplat_conv3x3_wino_bf16x3_ex_fwd")
        return y
    rc = lib.tsplat_conv3x3_wino_cat_f32_fwd(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(chans, ctypes.c_void_p),
                                             len(srcs), _lib.ptr(wino_pack_weight(weight)), _lib.ptr(pb),
                                             _lib.ptr(y), n, h, w, co, _WINO_ACT[act], _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_conv3x3_wino_cat_f32_fwd")
    return y


# bf16 implicit-GEMM 3x3 / 1x1 convolution (tsplat_conv2d_bf16_fwd) for the convolutions that run
# under bf16 autocast (config C3); "0" = MIOpen (A/B knob)
_CONV_BF16 = os.environ.get("TSPLAT_CONV_BF16", "1") != "0"
_BF16_PACKED: dict = {}


def conv_bf16_pack_weight(weight):
    """[cout, cin, k, k] (k = 1, 3) -> bf16 [ceil(cout / 32)][ceil(cin / 16)][k * k][64 lanes][8]
    (lane c + 32 h holds w[32 b + c][16 j + 8 h + 0..7][tap]), the A operand of
    tsplat_conv2d_bf16_fwd; cached per weight tensor version."""
    hit = _BF16_PACKED.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == weight._version:
        return hit[2]
    co, ci = weight.shape[:2]
    taps = weight[0, 0].numel()  # [co, ci, k, k] or a Conv1d's [co, ci, 1]
    cob, nk = (co + 31) // 32, (ci + 15) // 16
    w = torch.zeros((cob * 32, nk * 16, taps), dtype=torch.bfloat16, device=weight.device)
    w[:co, :ci] = weight.detach().reshape(co, ci, taps).to(torch.bfloat16)
    packed = w.view(cob, 32, nk, 2, 8, taps).permute(0, 2, 5, 3, 1, 4).contiguous()
    if len(_BF16_PACKED) > 512:
        for k in [k for k, v in _BF16_PACKED.items() if v[0]() is None]:
            del _BF16_PACKED[k]
    _BF16_PACKED[id(weight)] = (weakref.ref(weight), weight._version, packed)
    return packed


def _bf16_rounded_bias(bias):
    """fp32 copy of the bias rounded to bf16 (autocast's cast), cached per tensor version."""
    key = ("bias", id(bias))
    hit = _BF16_PACKED.get(key)
    if hit is not None and hit[0]() is bias and hit[1] == bias._version:
        return hit[2]
    rb = bias.detach().to(torch.bfloat16).float().contiguous()
    _BF16_PACKED[key] = (weakref.ref(bias), bias._version, rb)
    return rb


def conv_bf16_ok(x, weight, stride=1, padding=None, dilation=1, groups=1, extra=(), upsample: bool = False) -> bool:
    """True when conv2d(up(cat([x, *extra], 1)), weight) runs under bf16 autocast and fits
    tsplat_conv2d_bf16_fwd: 3x3 / padding 1 or 1x1 / padding 0, stride 1, NCHW contiguous fp32 or
    bf16 sources (any channel counts, dtypes may differ) with the convolved width a multiple of 8, at
    most 4 sources; up = optional nearest 2x upsample read in place."""
    if (not _CONV_BF16 or not x.is_cuda or not torch.is_autocast_enabled("cuda")
            or torch.get_autocast_dtype("cuda") != torch.bfloat16 or len(extra) > 3):
        return False
    for t in (x, *extra):
        if (t.dtype not in (torch.float32, torch.bfloat16) or t.dim() != 4 or not t.is_contiguous()
                or t.device != x.device or t.shape[0] != x.shape[0] or t.shape[2:] != x.shape[2:]
                or t.numel() >= 2 ** 31):
            return False
    # [co, ci, k, k] (k = 1, 3) or a 1x1 Conv1d's [co, ci, 1] (on a [n, c, 1, t] view of its input)
    if not ((weight.dim() == 4 and weight.shape[2] == weight.shape[3] and weight.shape[2] in (1, 3))
            or (weight.dim() == 3 and weight.shape[2] == 1)) or groups != 1:
        return False
    k = weight.shape[2]
    as_int = lambda v: v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else -1)
    if as_int(stride) != 1 or as_int(padding if padding is not None else k // 2) != k // 2 or as_int(dilation) != 1:
        return False
    n, _, h, w = x.shape
    if upsample:
        h, w = 2 * h, 2 * w
    ci = sum(t.shape[1] for t in (x, *extra))
    return weight.shape[1] == ci and w % 8 == 0 and n * max(weight.shape[0], ci) * h * w < 2 ** 31


def conv_bf16(x, weight, bias=None, act: str = "none", extra=(), upsample: bool = False):
    """act(conv2d(up(cat([x, *extra], 1)), weight, bias, 1, k // 2)) as autocast would compute it in
    bf16 (bf16-rounded sources, weights and bias, fp32 accumulation), output bf16 NCHW, in one
    tsplat_conv2d_bf16_fwd launch that reads the concatenation / nearest upsample in place."""
    import ctypes

    if not x.is_cuda:
        raise RuntimeError("transplat HIP ops need device tensors (no CPU path)")
    lib = _lib.load()
    srcs = (x, *extra)
    n, _, h, w = x.shape
    if upsample:
        h, w = 2 * h, 2 * w
    co, k = weight.shape[0], weight.shape[2]
    y = torch.empty((n, co, h, w), dtype=torch.bfloat16, device=x.device)
    pb = _bf16_rounded_bias(bias) if bias is not None else None
    ptrs = (ctypes.c_void_p * len(srcs))(*[_lib.ptr(t) for t in srcs])
    chans = (ctypes.c_int32 * len(srcs))(*[t.shape[1] for t in srcs])
    f32 = (ctypes.c_int32 * len(srcs))(*[int(t.dtype == torch.float32) for t in srcs])
    rc = lib.tsplat_conv2d_bf16_fwd(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(chans, ctypes.c_void_p),
                                    len(srcs), ctypes.cast(f32, ctypes.c_void_p),
                                    _lib.ptr(conv_bf16_pack_weight(weight)), _lib.ptr(pb), _lib.ptr(y), n, h, w,
                                    co, k, int(upsample), _ACTS[act], _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_conv2d_bf16_fwd")
    return y


def conv2d_nhwc_ok(x, weight) -> bool:
    """True when tsplat_conv2d_f32_nhwc_fwd takes conv(x, weight) (stride 1, padding k // 2) on the
    channels-last map x and (mode "auto") it is latency-bound (same rule as conv2d_direct_ok)."""
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.shape[1] == 1:
        return False
    return conv2d_direct_ok(x, weight, 1, weight.shape[-1] // 2)


def conv2d_nhwc(x, weight, bias=None, residual=None, relu_in: bool = False):
    """conv2d(relu(x) if relu_in else x, weight, bias, 1, k // 2) (+ residual) on channels-last
    fp32 maps, one exact-fp32 MFMA launch (tsplat_conv2d_f32_nhwc_fwd); returns channels-last."""
    lib = _lib.load()
    n, c, h, w = x.shape
    co, ci, k, _ = weight.shape
    if ci != c or not x.is_contiguous(memory_format=torch.channels_last) or x.dtype != torch.float32:
        raise ValueError("conv2d_nhwc needs a channels-last fp32 input matching the weight")
    y = torch.empty((n, co, h, w), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    res = None
    if residual is not None:
        res = residual.float().contiguous(memory_format=torch.channels_last)
        if res.shape != y.shape:
            raise ValueError(f"residual {tuple(res.shape)} != output {tuple(y.shape)}")
    tiles = ((n * h * w + 31) // 32) * ((co + 31) // 32)
    ksplit = 16
    while ksplit > 1 and (tiles * ksplit > 4096 or c // 2 < (2 if k == 3 else 16) * ksplit):
        ksplit //= 2
    pb = _f32(bias) if bias is not None else None
    rc = lib.tsplat_conv2d_f32_nhwc_fwd(_lib.ptr(x), c, _lib.ptr(conv_pack_weight(weight)), _lib.ptr(pb),
                                        _lib.ptr(res), _lib.ptr(y), n, h, w, co, k, int(relu_in), ksplit,
                                        _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_conv2d_f32_nhwc_fwd")
    return y


def upsample_bilinear_act(x, scale: int, bias=None, act: str = "none"):
    """act(interpolate(x, scale_factor=scale, mode="bilinear", align_corners=True) + bias[c]) in one
    pass (tsplat_upsample_bilinear_act_fwd), NCHW fp32."""
    lib = _lib.load()
    n, c, h, w = x.shape
    xf = _f32(x)
    y = torch.empty((n, c, h * scale, w * scale), dtype=torch.float32, device=x.device)
    rc = lib.tsplat_upsample_bilinear_act_fwd(_lib.ptr(xf), _lib.ptr(_f32(bias) if bias is not None else None),
                                              _lib.ptr(y), n, c, h, w, int(scale), _ACTS[act],
                                              _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_upsample_bilinear_act_fwd")
    return y


def qkv_attention_cf(qkv, heads: int, views: int = 1):
    """QKVAttentionLegacy (head dim 32, views folded into the tokens when views > 1):
    qkv [(v b), 3 * heads * 32, t] -> [(v b), heads * 32, t] in one launch
    (tsplat_qkv_attention_cf_fwd; no rearrange copies)."""
    lib = _lib.load()
    vb, width, t = qkv.shape
    ch = width // (3 * heads)
    if vb % views or ch * 3 * heads != width:
        raise ValueError(f"qkv {tuple(qkv.shape)} does not split into {views} views x {heads} heads")
    x = _f32(qkv)
    out = torch.empty((vb, heads * ch, t), dtype=torch.float32, device=qkv.device)
    rc = lib.tsplat_qkv_attention_cf_fwd(_lib.ptr(x), _lib.ptr(out), vb // views, heads, views, t, ch,
                                         float(ch ** -0.5), _lib.stream_ptr(qkv.device))
    _lib.check(rc, "tsplat_qkv_attention_cf_fwd")
    return out


def conv_nhwc_epilogue(conv, x, act: str = "none", res1=None, res2=None):
    """act(conv(x) + bias) (+ res1) (+ res2) on channels-last fp32 maps: the bias-free MIOpen
    convolution, then bias, activation and residuals in one pass (tsplat_bias_act_nhwc_fwd)."""
    import torch.nn.functional as F

    y = F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    cl = torch.channels_last
    if not y.is_contiguous(memory_format=cl):
        y = y.contiguous(memory_format=cl)
    rs = [r.contiguous(memory_format=cl) if r is not None else None for r in (res1, res2)]
    for r in rs:
        if r is not None and (r.shape != y.shape or r.dtype != torch.float32):
            raise ValueError(f"residual {tuple(r.shape)} does not match the output {tuple(y.shape)}")
    lib = _lib.load()
    rc = lib.tsplat_bias_act_nhwc_fwd(_lib.ptr(y), _lib.ptr(conv.bias), _lib.ptr(rs[0]), _lib.ptr(rs[1]),
                                      _lib.ptr(y), y.numel() // y.shape[1], y.shape[1], _ACTS[act],
                                      _lib.stream_ptr(y.device))
    _lib.check(rc, "tsplat_bias_act_nhwc_fwd")
    return y


def resize_bilinear_nhwc(x, size):
    """F.interpolate(x, size, mode="bilinear", align_corners=True) of a channels-last fp32 map in one
    launch (tsplat_resize_bilinear_nhwc_fwd); returns channels-last."""
    n, c, h, w = x.shape
    ho, wo = int(size[0]), int(size[1])
    if x.dtype != torch.float32 or not x.is_contiguous(memory_format=torch.channels_last) or c % 4:
        raise ValueError("resize_bilinear_nhwc needs a channels-last fp32 map with C % 4 == 0")
    y = torch.empty((n, c, ho, wo), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    lib = _lib.load()
    rc = lib.tsplat_resize_bilinear_nhwc_fwd(_lib.ptr(x), _lib.ptr(y), n, h, w, c, ho, wo, _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_resize_bilinear_nhwc_fwd")
    return y


def interpolate_bilinear_ac(x, size):
    """F.interpolate(x, size, mode="bilinear", align_corners=True). NCHW-contiguous fp32 device maps
    go through tsplat_resize_bilinear_nchw_fwd (one thread per output element; PyTorch's generic
    kernel serialises the N*C planes per output pixel: 240 us per call at C3's batch 8); anything
    else takes F.interpolate."""
    import torch.nn.functional as F

    size = (int(size[0]), int(size[1]))
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.is_contiguous()):
        return F.interpolate(x, size, mode="bilinear", align_corners=True)
    n, c, h, w = x.shape
    y = torch.empty((n, c, size[0], size[1]), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    rc = lib.tsplat_resize_bilinear_nchw_fwd(_lib.ptr(x), _lib.ptr(y), n * c, h, w, size[0], size[1],
                                             _lib.stream_ptr(x.device))
    _lib.check(rc, "tsplat_resize_bilinear_nchw_fwd")
    return y


def sh_rotation(rotations, d_sh: int):
    """[n, 3, 3] rotations -> [n, d_sh, d_sh] block-diagonal real-SH rotations (e3nn's
    wigner_D per degree, see misc/sh_rotation.py), one kernel launch."""
    from .misc.sh_rotation import x_basis_packed

    lib = _lib.load()
    rot = _f32(rotations.reshape(-1, 3, 3))
    n = rot.shape[0]
    out = torch.empty((n, d_sh, d_sh), device=rot.device)
    rc = lib.tsplat_sh_rotation_fwd(_lib.ptr(rot), _lib.ptr(x_basis_packed(rot.device)), _lib.ptr(out), n, d_sh,
                                    _lib.stream_ptr(rot.device))
    _lib.check(rc, "tsplat_sh_rotation_fwd")
    return out


def adapter_camera_consts(extrinsics, intrinsics, image_shape, d_sh: int):
    """The adapter's per-camera inputs, which depend on the cameras alone: (adapter_cameras, the
    per-camera Wigner-D blocks of sh_rotation) -- computed at the start of the step on a side stream
    by the encoder and handed to gaussian_adapter(camera_consts=...)."""
    return (adapter_cameras(extrinsics, intrinsics, image_shape),
            sh_rotation(extrinsics.reshape(-1, 4, 4)[:, :3, :3], d_sh))


def gaussian_adapter(raw, depths, densities, extrinsics, intrinsics, image_shape, scale_min: float,
                     scale_max: float, opacity_exponent: float = 1.0, gaussians_per_pixel: int = 1,
                     camera_consts=None):
    """Raw head output -> Gaussians (see oracle.gaussian_adapter). raw [B, V, HW, 9 + 3 d_sh];
    depths, densities [B, V, HW]; extrinsics [B, V, 4, 4]; intrinsics [B, V, 3, 3]
    -> means [B, V*HW, 3], covariances [B, V*HW, 3, 3], harmonics [B, V*HW, 3, d_sh], opacities [B, V*HW].
    camera_consts: adapter_camera_consts(...) if already computed."""
    lib = _lib.load()
    b, v, hw, r = raw.shape
    d_sh = (r - 9) // 3
    h, w = image_shape
    # the head's "(v b) c h w -> b v (h w) c" view of its NCHW output map is read in place
    # (strides of size-1 dimensions are arbitrary: compared only where the size is > 1)
    nchw = raw.dtype == torch.float32 and all(
        n == 1 or st == want for n, st, want in zip(raw.shape, raw.stride(), (r * hw, b * r * hw, 1, hw)))
    if not nchw:
        raw = _f32(raw)
    depths, densities = _f32(depths), _f32(densities)
    cams, shrot = camera_consts if camera_consts is not None else adapter_camera_consts(extrinsics, intrinsics,
                                                                                       image_shape, d_sh)
    dev = raw.device
    g = v * hw
    means = torch.empty((b, g, 3), device=dev)
    cov = torch.empty((b, g, 3, 3), device=dev)
    harm = torch.empty((b, g, 3, d_sh), device=dev)
    opac = torch.empty((b, g), device=dev)
    rc = lib.tsplat_gaussian_adapter_fwd(
        _lib.ptr(raw), _lib.ptr(depths), _lib.ptr(densities), _lib.ptr(cams), _lib.ptr(shrot), _lib.ptr(means),
        _lib.ptr(cov), _lib.ptr(harm), _lib.ptr(opac), b, v, h, w, r, d_sh, float(scale_min), float(scale_max),
        float(opacity_exponent), int(gaussians_per_pixel), int(nchw), _lib.stream_ptr(dev))
    _lib.check(rc, "tsplat_gaussian_adapter_fwd")
    return means, cov, harm, opac
