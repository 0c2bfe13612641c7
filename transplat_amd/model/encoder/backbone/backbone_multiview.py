"""CNN features -> camera encoding -> windowed position embedding -> multi-view transformer
(reference src/model/encoder/backbone/backbone_multiview.py:14-133)."""
from __future__ import annotations

import os

import torch
from einops import rearrange

from ...utils.cam_param_encoder import cam_param_encoder
from .multiview_transformer import MultiViewFeatureTransformer, stacked_views
from .unimatch import CNNEncoder, PositionEmbeddingSine, merge_splits, split_feature

_IMAGENET_MEAN = (0.485, 0.456, 0.406)
_IMAGENET_STD = (0.229, 0.224, 0.225)


_POSITION_CACHE: dict = {}
# the views' camera encodings in one call + the tiled window position ("0": per view, the A/B knob)
_BATCHED = os.environ.get("TSPLAT_BB_BATCHED", "1") == "1"


def _window_position(x, feature_channels):
    """Sine embedding of one window (constant per shape/device; cached)."""
    key = (tuple(x.shape), x.dtype, x.device, feature_channels)
    pos = _POSITION_CACHE.get(key)
    if pos is None:
        pos = PositionEmbeddingSine(num_pos_feats=feature_channels // 2)(x).to(x.dtype)
        _POSITION_CACHE[key] = pos
    return pos


def _tiled_window_position(x, attn_splits, feature_channels):
    """The window embedding of feature_add_position_list tiled over the attn_splits^2 windows of a
    full map, [1, C, H, W] (constant per shape; cached): x + it equals split -> + window position ->
    merge, element for element."""
    b, c, h, w = x.shape
    key = ("tiled", h, w, x.dtype, x.device, feature_channels, attn_splits)
    pos = _POSITION_CACHE.get(key)
    if pos is None:
        win = torch.empty((1, c, h // attn_splits, w // attn_splits), dtype=x.dtype, device=x.device)
        pos = _window_position(win, feature_channels).repeat(1, 1, attn_splits, attn_splits).contiguous()
        _POSITION_CACHE[key] = pos
    return pos


def feature_add_position_list(features_list, attn_splits, feature_channels):
    """(reference :14-34) add the sine embedding of one window to every window."""
    pos_enc = PositionEmbeddingSine(num_pos_feats=feature_channels // 2)
    if attn_splits > 1:
        features_splits = [split_feature(x, num_splits=attn_splits) for x in features_list]
        position = _window_position(features_splits[0], feature_channels)
        features_splits = [x + position for x in features_splits]
        return [merge_splits(x, num_splits=attn_splits) for x in features_splits]
    position = pos_enc(features_list[0])
    return [x + position for x in features_list]


class BackboneMultiview(torch.nn.Module):
    def __init__(self, feature_channels=128, num_transformer_layers=6, ffn_dim_expansion=4, num_head=1,
                 downscale_factor=8):
        super().__init__()
        self.feature_channels = feature_channels
        self.backbone = CNNEncoder(output_dim=feature_channels, num_output_scales=1 if downscale_factor == 8 else 0)
        self.transformer = MultiViewFeatureTransformer(num_layers=num_transformer_layers, d_model=feature_channels,
                                                       nhead=num_head, ffn_dim_expansion=ffn_dim_expansion)
        self.cam_param_encoder = cam_param_encoder(in_channels=128, mid_channels=128, embed_dims=128)
        self.register_buffer("img_mean", torch.tensor(_IMAGENET_MEAN), persistent=False)
        self.register_buffer("img_std", torch.tensor(_IMAGENET_STD), persistent=False)

    def normalize_images(self, images):
        shape = [*[1] * (images.dim() - 3), 3, 1, 1]
        return (images - self.img_mean.reshape(*shape)) / self.img_std.reshape(*shape)

    def extract_feature(self, images):
        b, v = images.shape[:2]
        features = self.backbone(rearrange(images, "b v c h w -> (b v) c h w"))[::-1]
        features_list = [[] for _ in range(v)]
        for feature in features:
            feature = rearrange(feature, "(b v) c h w -> b v c h w", b=b, v=v)
            for idx in range(v):
                features_list[idx].append(feature[:, idx])
        return features_list

    def forward(self, images, attn_splits=2, return_cnn_features=False, img2world=None):
        from ....misc.benchmarker import stage

        with stage(None, "backbone_cnn"):  # diagnostic sub-stage marks (TSPLAT_MARKS / TSPLAT_ROCTX)
            features_list = self.extract_feature(self.normalize_images(images))
        cur_features_list = [x[0] for x in features_list]
        cnn = torch.stack(cur_features_list, dim=1)  # [b, v, C, h, w]
        cnn_features = cnn if return_cnn_features else None
        b, v = cnn.shape[:2]
        if _BATCHED and attn_splits > 1 and cnn.shape[-2] % attn_splits == 0 and cnn.shape[-1] % attn_splits == 0:
            # all views in one camera-encoder call (per-sample ops: the same per view as the
            # reference's loop, reference :105-108) and the tiled window position added once
            enc = self.cam_param_encoder(cnn.flatten(0, 1), img2world.flatten(0, 1))
            enc = enc + _tiled_window_position(enc, attn_splits, self.feature_channels)
            cur_features_list = [t.contiguous() for t in enc.view(b, v, *enc.shape[1:]).unbind(1)]
        else:
            cur_features_list = [self.cam_param_encoder(f, img2world[:, v_id]) for v_id, f in enumerate(cur_features_list)]
            cur_features_list = feature_add_position_list(cur_features_list, attn_splits, self.feature_channels)
        with stage(None, "backbone_mvt"):
            cur_features_list = self.transformer(cur_features_list, attn_num_splits=attn_splits)
        features = stacked_views(cur_features_list)
        return [features, cnn_features]
