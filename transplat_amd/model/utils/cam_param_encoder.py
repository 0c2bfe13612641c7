"""Camera-parameter encoder (reference src/model/utils/cam_param_encoder.py:45-93): BN1d over the
16 img2world entries -> MLP -> SE gate on conv3x3-BN-ReLU(feature) -> 1x1 conv."""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from transplat_amd import kernels


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

    def _folded(self):
        """Eval-mode BatchNorms folded into their neighbours, cached per parameter version:
        reduce_conv's BatchNorm2d into the 3x3 conv's weight / bias, and the BatchNorm1d on the
        camera vector into context_mlp.fc1 (fc1(s x + c) = (W diag s) x + (W c + b))."""
        conv, bn2, fc1 = self.reduce_conv[0], self.reduce_conv[1], self.context_mlp.fc1
        params = (conv.weight, conv.bias, bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var, fc1.weight,
                  fc1.bias, self.bn.weight, self.bn.bias, self.bn.running_mean, self.bn.running_var)
        key = tuple((t.data_ptr(), t._version) for t in params)
        hit = self.__dict__.get("_fold")
        if hit is None or hit[0] != key:
            with torch.no_grad():
                s2 = bn2.weight / torch.sqrt(bn2.running_var + bn2.eps)
                w = (conv.weight * s2[:, None, None, None]).contiguous()
                b = ((conv.bias - bn2.running_mean) * s2 + bn2.bias).contiguous()
                s1 = self.bn.weight / torch.sqrt(self.bn.running_var + self.bn.eps)
                c1 = self.bn.bias - self.bn.running_mean * s1
                w1 = (fc1.weight * s1[None, :]).contiguous()
                b1 = (fc1.bias + fc1.weight @ c1).contiguous()
            hit = (key, w, b, w1, b1)
            self.__dict__["_fold"] = hit
        return hit[1:]

    def forward(self, feat, cam_params):
        vb = feat.shape[0]
        conv = self.reduce_conv[0]
        if (not self.training and feat.is_cuda and feat.dtype == torch.float32 and conv.bias is not None
                and not torch.is_autocast_enabled("cuda")
                and kernels.conv3x3_wino_ok(feat, conv.weight, conv.stride, conv.padding, conv.dilation,
                                            conv.groups, vs_miopen=True)):
            # inference: both BatchNorms folded, conv + bias + ReLU as one Winograd launch
            w, b, w1, b1 = self._folded()
            feat = kernels.conv3x3_wino(feat, w, b, act="relu")
            mlp = self.context_mlp
            context_se = mlp.fc2(mlp.act(F.linear(cam_params.reshape(vb, -1), w1, b1)))[..., None, None]
            return self.context_conv(self.context_se(feat, context_se))
        mlp_input = self.bn(cam_params.reshape(vb, -1))
        feat = self.reduce_conv(feat)
        context_se = self.context_mlp(mlp_input)[..., None, None]
        return self.context_conv(self.context_se(feat, context_se))
