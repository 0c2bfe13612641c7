"""UniMatch pieces used on the TranSplat path (reference src/model/encoder/backbone/unimatch/).

CNNEncoder (backbone.py:39-117) at 1/4 resolution, window split/merge (utils.py:34-81) and the
sine position embedding (position.py:6-43). Parameter names follow the reference so a
checkpoint's `encoder.backbone.backbone.*` keys load unchanged.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .... import kernels


class ResidualBlock(nn.Module):
    def __init__(self, in_planes, planes, norm_layer=nn.InstanceNorm2d, stride=1, dilation=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, dilation=dilation, padding=dilation,
                               stride=stride, bias=False)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, dilation=dilation, padding=dilation, bias=False)
        self.relu = nn.ReLU(inplace=True)
        self.norm1 = norm_layer(planes)
        self.norm2 = norm_layer(planes)
        if not stride == 1 or in_planes != planes:
            self.norm3 = norm_layer(planes)
        if stride == 1 and in_planes == planes:
            self.downsample = None
        else:
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward(self, x):
        if isinstance(self.norm1, nn.InstanceNorm2d) and not self.norm1.affine:
            # InstanceNorm + ReLU (+ residual + ReLU) as one GroupNorm-kernel launch each
            y = kernels.instance_norm(self.conv1(x), self.norm1.eps, "relu")
            if self.downsample is not None:
                x = kernels.instance_norm(self.downsample[0](x), self.norm3.eps)
            return kernels.instance_norm(self.conv2(y), self.norm2.eps, "relu", residual=x)
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class CNNEncoder(nn.Module):
    """conv7/s2 + 3 x 2 residual blocks (InstanceNorm) + 1x1 projection; 1/4 resolution when
    num_output_scales = 0 (reference backbone_multiview.py:49-54)."""

    def __init__(self, output_dim=128, norm_layer=nn.InstanceNorm2d, num_output_scales=1):
        super().__init__()
        if num_output_scales > 1:
            raise NotImplementedError("multi-scale trident branch is not on the TranSplat path")
        feature_dims = [64, 96, 128]
        self.conv1 = nn.Conv2d(3, feature_dims[0], kernel_size=7, stride=2, padding=3, bias=False)
        self.norm1 = norm_layer(feature_dims[0])
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = feature_dims[0]
        self.layer1 = self._make_layer(feature_dims[0], stride=1, norm_layer=norm_layer)
        self.layer2 = self._make_layer(feature_dims[1], stride=2, norm_layer=norm_layer)
        stride = 2 if num_output_scales == 1 else 1
        self.layer3 = self._make_layer(feature_dims[2], stride=stride, norm_layer=norm_layer)
        self.conv2 = nn.Conv2d(feature_dims[2], output_dim, 1, 1, 0)

    def _make_layer(self, dim, stride=1, dilation=1, norm_layer=nn.InstanceNorm2d):
        layer1 = ResidualBlock(self.in_planes, dim, norm_layer=norm_layer, stride=stride, dilation=dilation)
        layer2 = ResidualBlock(dim, dim, norm_layer=norm_layer, stride=1, dilation=dilation)
        self.in_planes = dim
        return nn.Sequential(layer1, layer2)

    def forward(self, x):
        if isinstance(self.norm1, nn.InstanceNorm2d) and not self.norm1.affine:
            x = kernels.instance_norm(self.conv1(x), self.norm1.eps, "relu")
        else:
            x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        return [self.conv2(x)]


def split_feature(feature, num_splits=2, channel_last=False):
    """[B, C, H, W] -> [B*K*K, C, H/K, W/K] (or channel-last), windows ordered (row, col)."""
    if channel_last:
        b, h, w, c = feature.size()
        return feature.view(b, num_splits, h // num_splits, num_splits, w // num_splits, c).permute(
            0, 1, 3, 2, 4, 5).reshape(b * num_splits * num_splits, h // num_splits, w // num_splits, c)
    b, c, h, w = feature.size()
    return feature.view(b, c, num_splits, h // num_splits, num_splits, w // num_splits).permute(
        0, 2, 4, 1, 3, 5).reshape(b * num_splits * num_splits, c, h // num_splits, w // num_splits)


def merge_splits(splits, num_splits=2, channel_last=False):
    if channel_last:
        b, h, w, c = splits.size()
        nb = b // num_splits // num_splits
        return splits.view(nb, num_splits, num_splits, h, w, c).permute(0, 1, 3, 2, 4, 5).contiguous().view(
            nb, num_splits * h, num_splits * w, c)
    b, c, h, w = splits.size()
    nb = b // num_splits // num_splits
    return splits.view(nb, num_splits, num_splits, c, h, w).permute(0, 3, 1, 4, 2, 5).contiguous().view(
        nb, c, num_splits * h, num_splits * w)


class PositionEmbeddingSine(nn.Module):
    """Normalised sine/cosine position embedding (reference position.py:6-43)."""

    def __init__(self, num_pos_feats=64, temperature=10000, normalize=True, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        self.scale = 2 * math.pi if scale is None else scale

    def forward(self, x):
        b, c, h, w = x.size()
        mask = torch.ones((b, h, w), device=x.device)
        y_embed = mask.cumsum(1, dtype=torch.float32)
        x_embed = mask.cumsum(2, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            y_embed = y_embed / (y_embed[:, -1:, :] + eps) * self.scale
            x_embed = x_embed / (x_embed[:, :, -1:] + eps) * self.scale
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=x.device)
        dim_t = self.temperature ** (2 * (dim_t // 2) / self.num_pos_feats)
        pos_x = x_embed[:, :, :, None] / dim_t
        pos_y = y_embed[:, :, :, None] / dim_t
        pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
        pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
        return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)
