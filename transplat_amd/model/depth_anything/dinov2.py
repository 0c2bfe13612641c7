"""DINOv2 ViT backbone as used by Depth-Anything-V2 (reference src/depth_anything_v2/dinov2.py,
dinov2_layers/*): patch 14, LayerScale blocks, bicubic position-embedding interpolation with the
0.1 offset, `get_intermediate_layers` with the final LayerNorm. Parameter names follow the
reference (`pretrained.{cls_token,pos_embed,mask_token,patch_embed.proj,blocks.{i}.{norm1,attn.
{qkv,proj},ls1.gamma,norm2,mlp.{fc1,fc2},ls2.gamma},norm}`). On the GPU, attention runs the
hand-written exact-fp32 MFMA kernel tsplat_mha_f32_fwd (kernels.mha) instead of xformers, and the
pre-norm residual steps run tsplat_residual_ln_fwd.
"""
from __future__ import annotations

import math
from functools import partial

import torch
import torch.nn.functional as F
from torch import nn

from ... import kernels


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size = (img_size, img_size)
        self.patch_size = (patch_size, patch_size)
        self.patches_resolution = (img_size // patch_size, img_size // patch_size)
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = nn.Identity()

    def forward(self, x):
        b, c, h, w = x.shape
        p = self.patch_size[0]
        if (x.is_cuda and x.dtype == torch.float32 and self.proj.weight.dtype == torch.float32
                and not torch.is_autocast_enabled("cuda") and h % p == 0 and w % p == 0):
            # stride = kernel: the patch projection is one [B*N, C*p*p] x [C*p*p, D] GEMM (hipBLASLt)
            # on the unfolded patches -- MIOpen's direct 14x14 stride-14 kernel took 63 us -- and
            # lands in the [B, N, D] token layout without the transpose
            patches = (x.reshape(b, c, h // p, p, w // p, p).permute(0, 2, 4, 1, 3, 5)
                       .reshape(b * (h // p) * (w // p), c * p * p))
            y = torch.addmm(self.proj.bias, patches, self.proj.weight.reshape(self.proj.weight.shape[0], -1).t())
            return self.norm(y.view(b, (h // p) * (w // p), -1))
        return self.norm(self.proj(x).flatten(2).transpose(1, 2))


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, bias=True):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)

    def forward(self, x, slabs: bool = False):
        """slabs=True (the fused block chain, whose residual step sums them): fc2 may return its
        split-K partial slabs [s, *x.shape] (kernels.gemm_x3)."""
        if (slabs and type(self.act) is nn.GELU and self.act.approximate == "none" and self.fc1.bias is not None
                and kernels.gemm_x3_ok(x, self.fc1.weight)):
            # bf16x3 dense mode: fc1 + bias + exact GELU and fc2 on the split-bf16 GEMM
            h = kernels.gemm_x3(x, self.fc1.weight, self.fc1.bias, act="gelu")
            return kernels.gemm_x3(h, self.fc2.weight, self.fc2.bias, ksplit=0)
        if type(self.act) is nn.GELU and self.act.approximate == "none":
            # bf16x3 dense mode: fc1 on hipBLASLt's emulated-xf32 GEMM + bias + exact GELU in one pass
            # (kernels.linear_xf32)
            if kernels.linear_xf32_ok(x, self.fc1.weight):
                return self.fc2(kernels.linear_xf32(x, self.fc1.weight, self.fc1.bias, act="gelu"))
        return self.fc2(self.act(self.fc1(x)))


class LayerScale(nn.Module):
    def __init__(self, dim, init_values=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))

    def forward(self, x):
        return x * self.gamma


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, proj_bias=True):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)

    def forward(self, x, slabs: bool = False):
        """slabs=True: proj may return split-K partial slabs (see Mlp.forward)."""
        b, n, c = x.shape
        if (slabs and c // self.num_heads == 64 and self.qkv.bias is not None and self.proj.bias is not None
                and kernels.gemm_x3_ok(x, self.qkv.weight)):
            # bf16x3 dense mode: both projections on the split-bf16 GEMM (bias in its epilogue), the
            # attention on the bf16x3 MFMA kernel straight from the [b, n, 3c] layout
            if kernels.mha_x3_ok(b * n):  # the projection writes the attention's hi / lo operands
                o = kernels.mha_presplit(kernels.gemm_x3(x, self.qkv.weight, self.qkv.bias, act="split"),
                                         self.num_heads, self.scale)
            else:
                o = kernels.mha(kernels.gemm_x3(x, self.qkv.weight, self.qkv.bias), self.num_heads, self.scale)
            return kernels.gemm_x3(o, self.proj.weight, self.proj.bias, ksplit=0)
        if x.dtype == torch.float32 and c // self.num_heads == 64 and not torch.is_autocast_enabled(x.device.type):
            # exact-fp32 MFMA attention straight from the qkv projection's layout; in bf16x3 mode the
            # projection runs without its bias (hipBLASLt's emulated-xf32 GEMM) and the attention
            # kernel folds the bias in (no separate bias pass)
            if self.qkv.bias is not None and kernels.linear_xf32_ok(x, self.qkv.weight):
                qkv = kernels.linear_xf32(x, self.qkv.weight)
                return self.proj(kernels.mha(qkv, self.num_heads, self.scale, bias=self.qkv.bias))
            return self.proj(kernels.mha(self.qkv(x), self.num_heads, self.scale))
        qkv = self.qkv(x).reshape(b, n, 3, self.num_heads, c // self.num_heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        x = F.scaled_dot_product_attention(q, k, v, scale=self.scale)
        return self.proj(x.transpose(1, 2).reshape(b, n, c))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True, proj_bias=True, ffn_bias=True,
                 init_values=None, norm_layer=nn.LayerNorm, act_layer=nn.GELU):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio), act_layer=act_layer, bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()

    def forward(self, x):
        x = x + self.ls1(self.attn(self.norm1(x)))
        return x + self.ls2(self.mlp(self.norm2(x)))


class DinoVisionTransformer(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4.0,
                 init_values=1.0, interpolate_offset=0.1, interpolate_antialias=False):
        super().__init__()
        norm_layer = partial(nn.LayerNorm, eps=1e-6)
        self.num_features = self.embed_dim = embed_dim
        self.num_tokens = 1
        self.n_blocks = depth
        self.num_heads = num_heads
        self.patch_size = patch_size
        self.num_register_tokens = 0
        self.interpolate_antialias = interpolate_antialias
        self.interpolate_offset = interpolate_offset
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=3, embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + self.num_tokens, embed_dim))
        self.blocks = nn.ModuleList([
            Block(embed_dim, num_heads, mlp_ratio=mlp_ratio, init_values=init_values, norm_layer=norm_layer)
            for _ in range(depth)])
        self.norm = norm_layer(embed_dim)
        self.head = nn.Identity()
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim))
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)

    def interpolate_pos_encoding(self, x, w, h):
        """(reference dinov2.py:185-217) bicubic resample of the 37x37 grid with the 0.1 offset.
        The result depends only on the weights and the input size, so it is cached (the bicubic
        kernel alone cost 2.3 ms per forward on MI355X); the key includes the parameter's version
        counter so a checkpoint load or in-place update invalidates it."""
        key = (w, h, x.dtype, x.device, self.pos_embed.data_ptr(), self.pos_embed._version)
        cached = getattr(self, "_pos_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        out = self._interpolate_pos_encoding(x, w, h)
        self._pos_cache = (key, out)
        return out

    def _interpolate_pos_encoding(self, x, w, h):
        previous_dtype = x.dtype
        npatch = x.shape[1] - 1
        n = self.pos_embed.shape[1] - 1
        if npatch == n and w == h:
            return self.pos_embed
        pos_embed = self.pos_embed.float()
        class_pos_embed = pos_embed[:, 0]
        patch_pos_embed = pos_embed[:, 1:]
        dim = x.shape[-1]
        w0 = w // self.patch_size + self.interpolate_offset
        h0 = h // self.patch_size + self.interpolate_offset
        sqrt_n = math.sqrt(n)
        sx, sy = float(w0) / sqrt_n, float(h0) / sqrt_n
        patch_pos_embed = F.interpolate(
            patch_pos_embed.reshape(1, int(sqrt_n), int(sqrt_n), dim).permute(0, 3, 1, 2),
            scale_factor=(sx, sy), mode="bicubic", antialias=self.interpolate_antialias)
        patch_pos_embed = patch_pos_embed.permute(0, 2, 3, 1).view(1, -1, dim)
        return torch.cat((class_pos_embed.unsqueeze(0), patch_pos_embed), dim=1).to(previous_dtype)

    def prepare_tokens(self, x):
        _, _, w, h = x.shape
        x = self.patch_embed(x)
        x = torch.cat((self.cls_token.expand(x.shape[0], -1, -1).to(x.dtype), x), dim=1)
        return x + self.interpolate_pos_encoding(x, w, h).to(x.dtype)

    def _fused_ok(self, x) -> bool:
        # fp32, or bf16 autocast (the linears then read the bf16 LayerNorm outputs directly)
        autocast = torch.is_autocast_enabled(x.device.type)
        ok_dtype = (x.dtype == torch.float32 and not autocast) or (
            autocast and torch.get_autocast_dtype(x.device.type) == torch.bfloat16 and x.is_cuda)
        return (ok_dtype and x.shape[-1] in (256, 512, 768, 1024)
                and all(isinstance(m, (LayerScale, nn.Identity)) for b in self.blocks for m in (b.ls1, b.ls2)))

    def _blocks_fused(self, x, take, norm: bool, on_output=None):
        """The block chain with every pre-norm residual step x = x + ls(y), h = norm_next(x) as ONE
        kernel (kernels.residual_ln) instead of mul + add + LayerNorm launches; same math."""
        gamma = lambda m: m.gamma if isinstance(m, LayerScale) else None
        blocks = self.blocks
        # bf16 autocast: the residual stream stays fp32 (as x + ls * y promotes it under autocast)
        # and the normalised rows are handed to the bf16 linears as bf16
        bf = torch.is_autocast_enabled(x.device.type)
        x = x.float()
        _, h = kernels.residual_ln(x, None, None, blocks[0].norm1, bf16_out=bf)
        outputs = []
        for i, blk in enumerate(blocks):
            x, h2 = kernels.residual_ln(x, blk.attn(h, slabs=True), gamma(blk.ls1), blk.norm2, bf16_out=bf)
            last = i + 1 == len(blocks)
            x, h = kernels.residual_ln(x, blk.mlp(h2, slabs=True), gamma(blk.ls2), self.norm if last else blocks[i + 1].norm1,
                                       bf16_out=bf)
            if i in take:
                if not norm:
                    outputs.append(x)
                else:  # the last block's step already produced self.norm(x)
                    outputs.append(h if last else kernels.residual_ln(x, None, None, self.norm, bf16_out=bf)[1])
                if on_output is not None:
                    on_output(len(outputs) - 1, outputs[-1])
        return outputs

    def get_intermediate_layers(self, x, n=4, reshape=False, return_class_token=False, norm=True,
                                on_output=None):
        """`on_output(k, tokens)` (not in the reference) is called as soon as the k-th taken layer's
        normed tokens [B, 1 + N, C] exist, so a consumer can start on them while the later blocks
        run (DepthAnythingV2.forward forks the DPT reassemble branches this way)."""
        x = self.prepare_tokens(x)
        take = range(len(self.blocks) - n, len(self.blocks)) if isinstance(n, int) else n
        if self._fused_ok(x):
            outputs = self._blocks_fused(x, take, norm, on_output)
        else:
            outputs = []
            for i, blk in enumerate(self.blocks):
                x = blk(x)
                if i in take:
                    outputs.append(self.norm(x) if norm else x)
                    if on_output is not None:
                        on_output(len(outputs) - 1, outputs[-1])
        class_tokens = [o[:, 0] for o in outputs]
        outputs = [o[:, 1:] for o in outputs]
        if return_class_token:
            return tuple(zip(outputs, class_tokens))
        return tuple(outputs)


def DINOv2(model_name: str) -> DinoVisionTransformer:  # noqa: N802 (reference factory name)
    cfg = {"vits": (384, 6), "vitb": (768, 12), "vitl": (1024, 16)}
    if model_name not in cfg:
        raise NotImplementedError(model_name)
    dim, heads = cfg[model_name]
    depth = 24 if model_name == "vitl" else 12
    return DinoVisionTransformer(img_size=518, patch_size=14, embed_dim=dim, depth=depth, num_heads=heads,
                                 mlp_ratio=4.0, init_values=1.0, interpolate_offset=0.1)
