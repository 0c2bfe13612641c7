"""Camera-parameter encoder (reference src/model/utils/cam_param_encoder.py:45-93): BN1d over the
16 img2world entries -> MLP -> SE gate on conv3x3-BN-ReLU(feature) -> 1x1 conv."""
from __future__ import annotations

from torch import nn


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.ReLU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x):
        return self.drop2(self.fc2(self.drop1(self.act(self.fc1(x)))))


class SELayer(nn.Module):
    def __init__(self, channels, act_layer=nn.ReLU, gate_layer=nn.Sigmoid):
        super().__init__()
        self.conv_reduce = nn.Conv2d(channels, channels, 1, bias=True)
        self.act1 = act_layer()
        self.conv_expand = nn.Conv2d(channels, channels, 1, bias=True)
        self.gate = gate_layer()

    def forward(self, x, x_se):
        x_se = self.conv_expand(self.act1(self.conv_reduce(x_se)))
        return x * self.gate(x_se)


class cam_param_encoder(nn.Module):  # noqa: N801  (reference class name kept for state_dict parity)
    def __init__(self, in_channels, mid_channels, embed_dims):
        super().__init__()
        self.embed_dims = embed_dims
        self.in_channels = in_channels
        self.mid_channels = mid_channels
        self.context_ch = embed_dims
        self.cam_param_len = 16
        self.reduce_conv = nn.Sequential(
            nn.Conv2d(in_channels, mid_channels, kernel_size=3, stride=1, padding=1),
            nn.BatchNorm2d(mid_channels),
            nn.ReLU(inplace=True),
        )
        self.context_conv = nn.Conv2d(mid_channels, self.context_ch, kernel_size=1, stride=1, padding=0)
        self.bn = nn.BatchNorm1d(self.cam_param_len)
        self.context_mlp = Mlp(self.cam_param_len, mid_channels, mid_channels)
        self.context_se = SELayer(mid_channels)

    def forward(self, feat, cam_params):
        vb = feat.shape[0]
        mlp_input = self.bn(cam_params.reshape(vb, -1))
        feat = self.reduce_conv(feat)
        context_se = self.context_mlp(mlp_input)[..., None, None]
        return self.context_conv(self.context_se(feat, context_se))
