"""CNN features -> camera encoding -> windowed position embedding -> multi-view transformer
(reference src/model/encoder/backbone/backbone_multiview.py:14-133)."""
from __future__ import annotations

import torch
from einops import rearrange

from ...utils.cam_param_encoder import cam_param_encoder
from .multiview_transformer import MultiViewFeatureTransformer
from .unimatch import CNNEncoder, PositionEmbeddingSine, merge_splits, split_feature

_IMAGENET_MEAN = (0.485, 0.456, 0.406)
_IMAGENET_STD = (0.229, 0.224, 0.225)


_POSITION_CACHE: dict = {}


def _window_position(x, feature_channels):
    """Sine embedding of one window (constant per shape/device; cached)."""
    key = (tuple(x.shape), x.dtype, x.device, feature_channels)
    pos = _POSITION_CACHE.get(key)
    if pos is None:
        pos = PositionEmbeddingSine(num_pos_feats=feature_channels // 2)(x).to(x.dtype)
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
        cnn_features = torch.stack(cur_features_list, dim=1) if return_cnn_features else None
        cur_features_list = [self.cam_param_encoder(f, img2world[:, v_id]) for v_id, f in enumerate(cur_features_list)]
        cur_features_list = feature_add_position_list(cur_features_list, attn_splits, self.feature_channels)
        with stage(None, "backbone_mvt"):
            cur_features_list = self.transformer(cur_features_list, attn_num_splits=attn_splits)
        features = torch.stack(cur_features_list, dim=1)
        return [features, cnn_features]
