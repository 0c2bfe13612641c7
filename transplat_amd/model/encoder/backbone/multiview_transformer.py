"""Multi-view swin transformer (reference src/model/encoder/backbone/multiview_transformer.py).

Same module tree and parameter names as the reference (`layers.{i}.self_attn.{q_proj,k_proj,
v_proj,merge,norm1}`, `layers.{i}.cross_attn_ffn.{...,mlp.{0,2},norm2}`) so checkpoints load;
the split-window attention (T2/T3 of SURVEY §8a: roll, partition, shifted mask, QK^T, softmax,
AV, merge, roll back) is ONE gfx950 kernel call (transplat_amd.kernels.window_attention).
"""
from __future__ import annotations

import os

import torch
from torch import nn

from .... import kernels


class TransformerLayer(nn.Module):
    """reference multiview_transformer.py:285-407 (swin, single head)."""

    def __init__(self, d_model=256, nhead=1, attention_type="swin", no_ffn=False, ffn_dim_expansion=4,
                 with_shift=False, add_per_view_attn=False, **kwargs):
        super().__init__()
        if nhead != 1 or attention_type != "swin" or add_per_view_attn:
            raise NotImplementedError("TranSplat uses single-head swin attention")
        self.dim = d_model
        self.nhead = nhead
        self.attention_type = attention_type
        self.no_ffn = no_ffn
        self.with_shift = with_shift
        self.q_proj = nn.Linear(d_model, d_model, bias=False)
        self.k_proj = nn.Linear(d_model, d_model, bias=False)
        self.v_proj = nn.Linear(d_model, d_model, bias=False)
        self.merge = nn.Linear(d_model, d_model, bias=False)
        self.norm1 = nn.LayerNorm(d_model)
        if not self.no_ffn:
            in_channels = d_model * 2
            self.mlp = nn.Sequential(
                nn.Linear(in_channels, in_channels * ffn_dim_expansion, bias=False),
                nn.GELU(),
                nn.Linear(in_channels * ffn_dim_expansion, d_model, bias=False),
            )
            self.norm2 = nn.LayerNorm(d_model)

    def _cat_weights(self, names: tuple[str, ...]) -> torch.Tensor:
        """[len(names) * d, d] concatenation of projection weights, cached until a weight changes
        (one fused launch computes q, k, v / k, v)."""
        ws = [getattr(self, n).weight for n in names]
        key = tuple((w.data_ptr(), w._version) for w in ws)
        cache = self.__dict__.setdefault("_wcat", {})
        hit = cache.get(names)
        if hit is None or hit[0] != key:
            hit = (key, torch.cat([w.detach() for w in ws], dim=0).contiguous())
            cache[names] = hit
        return hit[1]

    def _forward_fused(self, source, target, height, width, attn_num_splits, kv_shift: int = 0):
        """fp32 path: 4-5 kernels.fused_linear launches (exact fp32 MFMA, epilogues fused) around
        the attention kernel instead of ~12 PyTorch launches; same math as forward() below.
        kv_shift > 0: `target` is NOT view-swapped; query batch i reads the keys / values of its
        batch (i + kv_shift) % B (the swap is index arithmetic in the attention kernel)."""
        K = kernels
        kv_x3 = key = value = None
        # key views per query batch: 1 (self attention, the two-view pairing) or V - 1 (cross
        # attention with the other views stacked, target [B, V-1, L, C])
        kv_views = target.shape[1] if target.dim() == 4 else 1
        if source.dim() == 3 and K.attention_x3_ready(source.shape[0], height, width, kv_views, attn_num_splits):
            # bf16x3 attention: the k / v column blocks leave the projection as the kernel's bf16 hi / lo
            # operand (no fp32 k / v, no split pass); for V - 1 key views the buffer holds
            # [B, V-1, L, 128] per part, the layout the kernel indexes with key_views = V - 1
            if target is source:
                (query,), kv_x3 = K.linear_kv_x3(source, self._cat_weights(("q_proj", "k_proj", "v_proj")), 1)
            else:
                query = K.fused_linear(source, self.q_proj.weight)
                _, kv_x3 = K.linear_kv_x3(target, self._cat_weights(("k_proj", "v_proj")), 0)
        else:
            # bf16 window attention (C3 as stated): the projections written in bf16 directly
            od = torch.bfloat16 if K.projections_bf16(height, width, attn_num_splits) else torch.float32
            if target is source:
                query, key, value = K.fused_linear(source, self._cat_weights(("q_proj", "k_proj", "v_proj")),
                                                   split=True, out_dtype=od)
            else:
                query = K.fused_linear(source, self.q_proj.weight, out_dtype=od)
                key, value = K.fused_linear(target, self._cat_weights(("k_proj", "v_proj")), split=True, out_dtype=od)
        ln1 = (self.norm1.weight, self.norm1.bias, self.norm1.eps)
        x3 = {"kv_x3": kv_x3, "kv_views": kv_views} if kv_x3 is not None else {}
        if self.no_ffn:
            return K.attention_merge(query, key, value, height, width, attn_num_splits, self.with_shift,
                                     self.merge.weight, ln1, residual=source, kv_shift=kv_shift, **x3)
        message = K.attention_merge(query, key, value, height, width, attn_num_splits, self.with_shift,
                                    self.merge.weight, ln1, kv_shift=kv_shift, **x3)
        # mlp[0] is the one large plain GEMM of the layer (8192 x 256 x 1024 at b = 1): in the bf16x3
        # mode on the split-bf16 GEMM (26.6 us; hipBLASLt exact fp32 35.8), else hipBLASLt (103 TF,
        # above linear.hip's 66); its GELU moves into mlp[2]'s load
        cat = torch.cat([source, message], dim=-1)
        w0 = self.mlp[0].weight
        hidden = K.gemm_x3(cat, w0, self.mlp[0].bias) if K.gemm_x3_ok(cat, w0) else self.mlp[0](cat)
        ln2 = (self.norm2.weight, self.norm2.bias, self.norm2.eps)
        return K.fused_linear(hidden, self.mlp[2].weight, ln=ln2, residual=source, gelu_in=True)

    def forward(self, source, target, height=None, width=None, attn_num_splits=None, **kwargs):
        # source [B, L, C]; target [B, L, C] (self) or [B, V-1, L, C] (cross)
        if source.dtype == torch.float32 and self.dim == 128 and not torch.is_autocast_enabled(source.device.type):
            return self._forward_fused(source, target, height, width, attn_num_splits)
        ln128 = self._ln128_ok(source)
        if ln128:
            # bf16 dense mode: the fp32 residual stream is cast once per layer (autocast would cast
            # it again for every projection that reads it, and for the FFN's concat)
            source16 = source.to(torch.bfloat16)
            target16 = source16 if target is source else target.to(torch.bfloat16)
        else:
            source16, target16 = source, target
        query = self.q_proj(source16)
        key = self.k_proj(target16)
        value = self.v_proj(target16)
        message = kernels.window_attention(query, key, value, height, width, attn_num_splits, self.with_shift)
        if ln128:
            # bf16 dense mode: each LayerNorm (+ the `source + message` residual) as one kernel on
            # the bf16 linear output (autocast would run PyTorch's LayerNorm in fp32 between casts)
            if self.no_ffn:
                return kernels.layer_norm128(self.merge(message), self.norm1, residual=source,
                                             out_dtype=torch.float32)
            message = kernels.layer_norm128(self.merge(message), self.norm1, out_dtype=torch.bfloat16)
            hidden = self.mlp(torch.cat([source16, message], dim=-1))
            return kernels.layer_norm128(hidden, self.norm2, residual=source, out_dtype=torch.float32)
        message = self.norm1(self.merge(message))
        if not self.no_ffn:
            message = self.norm2(self.mlp(torch.cat([source, message], dim=-1)))
        return source + message

    def _ln128_ok(self, source) -> bool:
        return (self.dim == 128 and source.is_cuda and torch.is_autocast_enabled(source.device.type)
                and torch.get_autocast_dtype(source.device.type) == torch.bfloat16 and kernels.BF16_NORMS)


class TransformerBlock(nn.Module):
    """self attention + cross attention + FFN (reference :410-492)."""

    def __init__(self, d_model=256, nhead=1, attention_type="swin", ffn_dim_expansion=4, with_shift=False,
                 add_per_view_attn=False, no_cross_attn=False, **kwargs):
        super().__init__()
        if no_cross_attn:
            raise NotImplementedError("TranSplat always uses cross-view attention")
        self.no_cross_attn = no_cross_attn
        self.self_attn = TransformerLayer(d_model=d_model, nhead=nhead, attention_type=attention_type,
                                          no_ffn=True, ffn_dim_expansion=ffn_dim_expansion, with_shift=with_shift)
        self.cross_attn_ffn = TransformerLayer(d_model=d_model, nhead=nhead, attention_type=attention_type,
                                               ffn_dim_expansion=ffn_dim_expansion, with_shift=with_shift,
                                               add_per_view_attn=add_per_view_attn)

    def forward(self, source, target, height=None, width=None, attn_num_splits=None, **kwargs):
        source = self.self_attn(source, source, height=height, width=width, attn_num_splits=attn_num_splits)
        return self.cross_attn_ffn(source, target, height=height, width=width, attn_num_splits=attn_num_splits)

    def forward_pair(self, x, height, width, attn_num_splits, kv_shift: int):
        """Two views stacked [v0; v1] in x (fp32 fused path): self attention, then cross attention
        against the other view as a key-batch shift instead of a swapped copy."""
        # the cross layer's keys / values come from the block INPUT (reference batch_features runs
        # between blocks, :624-628), its queries from the self-attention output
        y = self.self_attn._forward_fused(x, x, height, width, attn_num_splits)
        return self.cross_attn_ffn._forward_fused(y, x, height, width, attn_num_splits, kv_shift=kv_shift)


_ONE_COPY = os.environ.get("TSPLAT_MVT_ONE_COPY", "1") == "1"  # A/B knob for the single-copy output


def stacked_views(features):
    """torch.stack(features, dim=1), without a copy when the views already are the unbound views
    of one contiguous [b, v, ...] tensor (MultiViewFeatureTransformer's two-view output)."""
    base = features[0]._base
    if (base is not None and base.is_contiguous() and base.dim() == features[0].dim() + 1
            and base.shape[1] == len(features)
            and all(f._base is base and f.data_ptr() == base[:, i].data_ptr() and f.shape == base[:, i].shape
                    and f.stride() == base[:, i].stride() for i, f in enumerate(features))):
        return base
    return torch.stack(features, dim=1)


def batch_features(features):
    """(reference :495-515) queries [N*B, ...] and the other N-1 views [N*B, N-1, ...]."""
    q, kv = [], []
    for i in range(len(features)):
        x = list(features)
        q.append(x.pop(i))
        kv.append(torch.stack(x, dim=1))
    return torch.cat(q, dim=0), torch.cat(kv, dim=0)


class MultiViewFeatureTransformer(nn.Module):
    """6 blocks of self + cross window attention (reference :518-630); odd blocks shifted."""

    def __init__(self, num_layers=6, d_model=128, nhead=1, attention_type="swin", ffn_dim_expansion=4,
                 add_per_view_attn=False, no_cross_attn=False, **kwargs):
        super().__init__()
        self.attention_type = attention_type
        self.d_model = d_model
        self.nhead = nhead
        self.layers = nn.ModuleList([
            TransformerBlock(d_model=d_model, nhead=nhead, attention_type=attention_type,
                             ffn_dim_expansion=ffn_dim_expansion, with_shift=(attention_type == "swin" and i % 2 == 1),
                             add_per_view_attn=add_per_view_attn, no_cross_attn=no_cross_attn)
            for i in range(num_layers)
        ])
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def forward(self, multi_view_features, attn_num_splits=None, **kwargs):
        b, c, h, w = multi_view_features[0].shape
        assert self.d_model == c
        num_views = len(multi_view_features)
        if not attn_num_splits or attn_num_splits <= 1:
            raise NotImplementedError("TranSplat runs split-window attention (multiview_trans_attn_split=2)")
        if (num_views == 2 and c == 128 and multi_view_features[0].dtype == torch.float32
                and not torch.is_autocast_enabled(multi_view_features[0].device.type)):
            # two views: batch_features' concat0 after each block is the block output itself and
            # concat1 its view swap, so the layers pair query batch i with key batch (i + b) % 2b
            x = torch.cat(multi_view_features, dim=0).reshape(2 * b, c, -1).permute(0, 2, 1).contiguous()
            for layer in self.layers:
                x = layer.forward_pair(x, h, w, attn_num_splits, kv_shift=b)
            # both views' NCHW maps in ONE permute copy, as views of a [b, v, c, h, w] tensor (the
            # backbone stacks them without another copy, see stacked_views)
            if not _ONE_COPY:
                return [f.view(b, h, w, c).permute(0, 3, 1, 2).contiguous() for f in x.chunk(chunks=2, dim=0)]
            stacked = x.view(2, b, h, w, c).permute(1, 0, 4, 2, 3).contiguous()
            return list(stacked.unbind(1))
        concat0, concat1 = batch_features(multi_view_features)
        concat0 = concat0.reshape(num_views * b, c, -1).permute(0, 2, 1)  # [N*B, HW, C]
        concat1 = concat1.reshape(num_views * b, num_views - 1, c, -1).permute(0, 1, 3, 2)  # [N*B, N-1, HW, C]
        for i, layer in enumerate(self.layers):
            concat0 = layer(concat0, concat1, height=h, width=w, attn_num_splits=attn_num_splits)
            if i < len(self.layers) - 1:
                concat0, concat1 = batch_features(list(concat0.chunk(chunks=num_views, dim=0)))
        features = concat0.chunk(chunks=num_views, dim=0)
        return [f.view(b, h, w, c).permute(0, 3, 1, 2).contiguous() for f in features]
