"""LDM-style 2-D U-Net with cross-view self-attention, as configured by DepthPredictorTrans
(reference src/model/encoder/matching/ldm_unet/{unet.py:589-1144, util.py}).

Only the configuration the depth predictor instantiates is built: postnorm ResBlocks, conv
down/up-sampling, legacy QKV attention at the requested resolutions with views folded into the
token axis, middle block = ResBlock, Identity, ResBlock. Module indices and parameter names
follow the reference (`input_blocks.{i}.{j}`, `middle_block.{0,2}`, `output_blocks.{i}.{j}`,
`out.{0,1}`) so checkpoint keys load. The latency-bound low-resolution convolutions run as a direct
fp32 MFMA kernel reading the skip concat / nearest upsample in place (kernels.conv2d_direct), the
rest and the GEMMs on MIOpen / hipBLASLt; every
GroupNorm runs as one fused gfx950 kernel pair together with the activation and residual add
that follow it in the reference's module chain (kernels.group_norm).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F
from einops import rearrange
from torch import nn

from .... import kernels

_ACT_OF = {nn.SiLU: "silu", nn.GELU: "gelu"}
_GEMM_1X1 = os.environ.get("TSPLAT_UNET_GEMM1X1", "1") != "0"  # A/B knob


def gn_act(norm: nn.GroupNorm, x, act: str = "none", residual=None, pre_bias=None):
    """act(norm(x + pre_bias)) [+ residual] in one fused kernel, computed in fp32 and returned in
    x's dtype (GroupNorm32 semantics: the reference normalises in float and casts back)."""
    y = kernels.group_norm(x, norm.num_groups, norm.weight, norm.bias, norm.eps, act, residual, pre_bias)
    return y.type(x.dtype)


# the output blocks' skip concatenation read in place by both ResBlock convolutions in the bf16x3
# mode (round 6; TSPLAT_UNET_CAT_FREE=0: materialised once, the A/B knob)
_CAT_FREE = os.environ.get("TSPLAT_UNET_CAT_FREE", "1") == "1"


def _direct(conv: nn.Module, x, x2=None, upsample: bool = False) -> bool:
    """Whether conv(cat([x, x2])) runs as the direct kernel (kernels.conv2d_direct_ok)."""
    if not (isinstance(conv, nn.Conv2d) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.stride[0] == conv.stride[1]):
        return False
    c2 = x2.shape[1] if x2 is not None else 0
    return kernels.conv2d_direct_ok(x, conv.weight, conv.stride[0], conv.padding, c2=c2, upsample=upsample)


def conv(conv: nn.Module, x, x2=None, upsample: bool = False, bias: bool = True):
    """conv(cat([x, x2], 1) (nearest-upsampled 2x if upsample)) [+ bias]. The latency-bound 2-D
    convolutions of the low-resolution levels run as one direct fp32 MFMA kernel that reads the
    concat / upsample in place (kernels.conv2d_direct); the rest materialise them and run MIOpen."""
    b = conv.bias if bias else None
    extra = (x2,) if x2 is not None else ()
    if (isinstance(conv, nn.Conv2d) and conv.padding_mode == "zeros"
            and kernels.conv_bf16_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, extra,
                                     upsample)):
        # bf16 autocast (C3): 3x3 / 1x1 on bf16 MFMA, the concat / upsample read in place
        return kernels.conv_bf16(x, conv.weight, b, extra=extra, upsample=upsample)
    if (isinstance(conv, nn.Conv1d) and x2 is None and not upsample and conv.kernel_size == (1,)
            and conv.stride == (1,) and conv.groups == 1 and x.dim() == 3
            and kernels.conv_bf16_ok(x.unsqueeze(2), conv.weight)):
        # the attention blocks' qkv / proj_out under bf16 autocast: a 1x1 over [n, c, t] viewed as a
        # [n, c, 1, t] map (MIOpen ran the 1-D form as im2col + GEMM)
        return kernels.conv_bf16(x.unsqueeze(2), conv.weight, b).squeeze(2)
    if _direct(conv, x, x2, upsample):
        return kernels.conv2d_direct(x, conv.weight, b, conv.stride[0], x2=x2, upsample=upsample)
    if (isinstance(conv, nn.Conv1d) and x2 is None and not upsample and conv.kernel_size == (1,)
            and conv.stride == (1,) and conv.groups == 1 and x.dim() == 3
            and kernels.conv2d_direct_ok(x.unsqueeze(-1), conv.weight)):
        # the attention blocks' qkv / proj_out: a 1x1 over [n, c, t] viewed as [n, c, t, 1]
        return kernels.conv2d_direct(x.unsqueeze(-1), conv.weight, b).squeeze(-1)
    if (isinstance(conv, nn.Conv2d) and not upsample
            and kernels.conv3x3_wino_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, extra)):
        return kernels.conv3x3_wino(x, conv.weight, b, extra=extra)  # the skip concat read in place
    if x2 is not None:
        x = torch.cat([x, x2], dim=1)
    if upsample:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    if isinstance(conv, nn.Conv2d) and kernels.conv3x3_wino_ok(x, conv.weight, conv.stride, conv.padding,
                                                               conv.dilation, conv.groups):
        return kernels.conv3x3_wino(x, conv.weight, b)
    if (_GEMM_1X1 and isinstance(conv, nn.Conv2d) and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.groups == 1
            and conv.padding == (0, 0) and x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32
            and not torch.is_autocast_enabled("cuda")):
        # a full-resolution 1x1 (the 256^2 skip convolutions) as one batched GEMM per image,
        # [cout, cin] x [cin, h*w]: HBM-bound ~10 us where MIOpen's NCHW 1x1 kernel took 45 us
        n, ci, h, w = x.shape
        co = conv.weight.shape[0]
        wm = conv.weight.view(co, ci).expand(n, co, ci)
        xm = x.contiguous().view(n, ci, h * w)
        y = torch.baddbmm(b.view(1, co, 1), wm, xm) if b is not None else torch.bmm(wm, xm)
        return y.view(n, co, h, w)
    if isinstance(conv, nn.Conv2d):
        return kernels.conv2d_fallback(x, conv.weight, b, conv.stride, conv.padding, conv.dilation, conv.groups)
    return F.conv1d(x, conv.weight, b, conv.stride, conv.padding, conv.dilation, conv.groups)


def conv_nobias(conv_mod: nn.Module, x, x2=None):
    """The convolution without its bias (the following fused GroupNorm adds it)."""
    return conv(conv_mod, x, x2, bias=False)


def conv_gn_act(conv_mod: nn.Module, norm: nn.GroupNorm, x, act: str = "none", residual=None, x2=None):
    """conv -> GroupNorm -> act (-> + residual) with the conv bias folded into the norm kernel."""
    if conv_mod.bias is None:
        return gn_act(norm, conv(conv_mod, x, x2), act, residual)
    return gn_act(norm, conv_nobias(conv_mod, x, x2), act, residual, pre_bias=conv_mod.bias)


def run_sequential(seq: nn.Sequential, x):
    """Run an nn.Sequential, fusing each GroupNorm with a SiLU / GELU that directly follows it."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, (nn.Conv1d, nn.Conv2d)) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.GroupNorm):
            nxt = mods[i + 2] if i + 2 < len(mods) else None
            act = _ACT_OF.get(type(nxt)) if nxt is not None else None
            if isinstance(nxt, nn.GELU) and nxt.approximate != "none":
                act = None
            x = conv_gn_act(m, mods[i + 1], x, act or "none")
            i += 3 if act else 2
            continue
        if isinstance(m, nn.GroupNorm):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            act = _ACT_OF.get(type(nxt)) if nxt is not None else None
            if isinstance(nxt, nn.GELU) and nxt.approximate != "none":
                act = None
            x = gn_act(m, x, act or "none")
            i += 2 if act else 1
            continue
        x = m(x)
        i += 1
    return x


class GroupNorm32(nn.GroupNorm):
    def forward(self, x):
        return gn_act(self, x)


def normalization(channels):
    """GroupNorm8 when channels % 8 == 0 else GroupNorm4 (reference util.py:189-208)."""
    return GroupNorm32(8 if channels % 8 == 0 else 4, channels)


class ResBlock(nn.Module):
    """postnorm residual block (reference unet.py:177-300): conv-GN-SiLU, conv-GN-SiLU, skip."""

    def __init__(self, channels, out_channels=None, kernel_size=3):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        pad = (kernel_size - 1) // 2
        self.in_layers = nn.Sequential(
            nn.Conv2d(channels, self.out_channels, kernel_size, padding=pad), normalization(self.out_channels),
            nn.SiLU())
        self.out_layers = nn.Sequential(
            nn.Conv2d(self.out_channels, self.out_channels, kernel_size, padding=pad),
            normalization(self.out_channels), nn.SiLU())
        self.skip_connection = (nn.Identity() if self.out_channels == channels
                                else nn.Conv2d(channels, self.out_channels, 1))

    def _concat_free(self, x, x2) -> bool:
        """bf16x3 mode, a Winograd / few-channel in_layers conv: both convolutions read cat([x, x2])
        in place (the 3x3 as a two-source launch, a 1x1 skip on the two-source direct kernel)."""
        c, sk = self.in_layers[0], self.skip_connection
        if not (_CAT_FREE and kernels.split_mode() and isinstance(c, nn.Conv2d)
                and kernels.conv3x3_wino_ok(x, c.weight, c.stride, c.padding, c.dilation, c.groups, (x2,))):
            return False
        return isinstance(sk, nn.Identity) or (
            isinstance(sk, nn.Conv2d) and sk.kernel_size == (1, 1) and sk.stride == (1, 1) and sk.groups == 1
            and kernels.conv2d_direct_ok(x, sk.weight, 1, sk.padding, c2=x2.shape[1], force=True))

    def forward(self, x, x2=None):
        # skip + SiLU(GN(conv(SiLU(GN(conv(x)))))): both GN + SiLU pairs and the residual fused;
        # x2: the output blocks' skip input, x = cat([x, x2], 1) without materialising the concat
        # where the convolutions read it in place
        cat_free = False
        if x2 is not None and not _direct(self.in_layers[0], x, x2):
            cat_free = self._concat_free(x, x2)
            if not cat_free:
                x, x2 = torch.cat([x, x2], dim=1), None  # materialised once for both convolutions
        h = conv_gn_act(self.in_layers[0], self.in_layers[1], x, "silu", x2=x2)
        if isinstance(self.skip_connection, nn.Identity):
            skip = x if x2 is None else (x, x2)  # the concat read in place by the norm's residual add
        elif cat_free and not _direct(self.skip_connection, x, x2):
            sk = self.skip_connection
            skip = kernels.conv2d_direct(x, sk.weight, sk.bias, 1, x2=x2)
        else:
            skip = conv(self.skip_connection, x, x2)
        return conv_gn_act(self.out_layers[0], self.out_layers[1], h, "silu", residual=skip)


class QKVAttentionLegacy(nn.Module):
    """heads split before q/k/v; views folded into tokens ((v b) n t -> b n (v t))
    (reference unet.py:510-552)."""

    def __init__(self, n_heads, n_frames=2, use_cross_view_self_attn=False):
        super().__init__()
        self.n_heads = n_heads
        self.n_frames = n_frames
        self.use_cross_view_self_attn = use_cross_view_self_attn

    def forward(self, qkv):
        width = qkv.shape[1]
        if qkv.is_cuda and width // (3 * self.n_heads) == 32 and (
                qkv.dtype == torch.float32 or torch.is_autocast_enabled("cuda")):
            # one kernel reading / writing the (v b) layout in place (kernels.qkv_attention_cf); under
            # bf16 autocast the qkv projection's bf16 output is widened once and the attention runs in
            # fp32 (the reference's einsum path: bf16 products, fp32 softmax; 8 launches)
            return kernels.qkv_attention_cf(qkv.float(), self.n_heads,
                                            self.n_frames if self.use_cross_view_self_attn else 1)
        if self.use_cross_view_self_attn:
            qkv = rearrange(qkv, "(v b) n t -> b n (v t)", v=self.n_frames)
        bs, width, length = qkv.shape
        ch = width // (3 * self.n_heads)
        q, k, v = qkv.reshape(bs * self.n_heads, ch * 3, length).split(ch, dim=1)
        scale = 1 / math.sqrt(math.sqrt(ch))
        weight = torch.einsum("bct,bcs->bts", q * scale, k * scale)
        weight = torch.softmax(weight.float(), dim=-1).type(weight.dtype)
        a = torch.einsum("bts,bcs->bct", weight, v).reshape(bs, -1, length)
        if self.use_cross_view_self_attn:
            a = rearrange(a, "b n (v t) -> (v b) n t", v=self.n_frames)
        return a


class AttentionBlock(nn.Module):
    """postnorm self-attention block (reference unet.py:306-370)."""

    def __init__(self, channels, num_head_channels=32, num_frames=2, use_cross_view_self_attn=False):
        super().__init__()
        self.channels = channels
        self.num_heads = channels // num_head_channels
        self.qkv = nn.Conv1d(channels, channels * 3, 1)
        self.attention = QKVAttentionLegacy(self.num_heads, n_frames=num_frames,
                                            use_cross_view_self_attn=use_cross_view_self_attn)
        self.proj_out = nn.Conv1d(channels, channels, 1)
        self.norm = normalization(channels)

    def forward(self, x):
        b, c, *spatial = x.shape
        x = x.reshape(b, c, -1)
        h = self.attention(conv(self.qkv, x))
        return conv_gn_act(self.proj_out, self.norm, h, residual=x).reshape(b, c, *spatial)


class Downsample(nn.Module):
    def __init__(self, channels, out_channels=None):
        super().__init__()
        self.channels = channels
        self.op = nn.Conv2d(channels, out_channels or channels, 3, stride=2, padding=1)

    def forward(self, x):
        return conv(self.op, x)


class Upsample(nn.Module):
    def __init__(self, channels, out_channels=None):
        super().__init__()
        self.channels = channels
        self.conv = nn.Conv2d(channels, out_channels or channels, 3, padding=1)

    def forward(self, x):
        return conv(self.conv, x, upsample=True)


class UNetModel(nn.Module):
    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks, attention_resolutions,
                 dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True, dims=2, postnorm=False,
                 num_head_channels=-1, num_frames=2, use_cross_view_self_attn=False, **kwargs):
        super().__init__()
        if dims != 2 or not postnorm or not conv_resample or num_head_channels <= 0:
            raise NotImplementedError("only the DepthPredictorTrans configuration is built")
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        attn = lambda ch: AttentionBlock(ch, num_head_channels=num_head_channels, num_frames=num_frames,
                                         use_cross_view_self_attn=use_cross_view_self_attn)
        self.input_blocks = nn.ModuleList([nn.Sequential(nn.Conv2d(in_channels, model_channels, 3, padding=1))])
        input_block_chans = [model_channels]
        ch = model_channels
        ds = 1
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks):
                layers = [ResBlock(ch, out_channels=mult * model_channels)]
                ch = mult * model_channels
                if ds in attention_resolutions:
                    layers.append(attn(ch))
                self.input_blocks.append(nn.Sequential(*layers))
                input_block_chans.append(ch)
            if level != len(channel_mult) - 1:
                self.input_blocks.append(nn.Sequential(Downsample(ch, out_channels=ch)))
                input_block_chans.append(ch)
                ds *= 2
        self.middle_block = nn.Sequential(ResBlock(ch), nn.Identity(), ResBlock(ch))
        self.output_blocks = nn.ModuleList([])
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks + 1):
                ich = input_block_chans.pop()
                layers = [ResBlock(ch + ich, out_channels=model_channels * mult)]
                ch = model_channels * mult
                if ds in attention_resolutions:
                    layers.append(attn(ch))
                if level and i == num_res_blocks:
                    layers.append(Upsample(ch, out_channels=ch))
                    ds //= 2
                self.output_blocks.append(nn.Sequential(*layers))
        self.out = nn.Sequential(nn.Conv2d(model_channels, out_channels, 3, padding=1), normalization(out_channels),
                                 nn.SiLU())

    def forward(self, x, timesteps=None, context=None, y=None, **kwargs):
        hs = []
        h = x
        for module in self.input_blocks:
            h = module(h)
            hs.append(h)
        h = self.middle_block(h)
        for module in self.output_blocks:
            # ResBlock(cat([h, skip])): the concat is read in place by its convolutions
            mods = list(module)
            h = mods[0](h, hs.pop())
            for m in mods[1:]:
                h = m(h)
        return run_sequential(self.out, h)
