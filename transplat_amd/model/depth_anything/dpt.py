"""Depth-Anything-V2 DPT head + model (reference src/depth_anything_v2/dpt.py:38-184,
util/blocks.py). Returns (relative depth [B, H, W], the 64-channel output_conv1 feature) exactly
as the reference forward does; parameter names match (`depth_head.{projects,resize_layers,
scratch.{layer*_rn,refinenet*,output_conv*}}`)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn


from ... import kernels, streams
from .dinov2 import DINOv2

# The token maps enter the DPT as channels-last views (permute of [B, N, C]); the whole conv chain
# then runs MIOpen's NHWC kernels, measured ~4% faster end-to-end than an NCHW copy up front. The
# conv weights are laid out channels-last once (first forward) so torch stops re-laying them out
# on every call.
_DPT_CL_WEIGHTS = os.environ.get("TSPLAT_DPT_CL_WEIGHTS", "1") != "0"
# Opt-in: "1" runs the latency-bound DPT convolutions (ResidualConvUnits <= 36^2, out_convs) as the
# channels-last direct kernel (kernels.conv2d_nhwc, ReLU / bias / residual fused), "rcu" only the
# units. Measured 2.0 % ("1") and 1.3 % ("rcu") SLOWER end to end than MIOpen's NHWC kernels: the
# kernel's pixel-per-lane B gathers touch 32 cache lines per load on a channels-last map. Default
# "0" (MIOpen) until the operand is staged through LDS.
_DPT_DIRECT = os.environ.get("TSPLAT_DPT_DIRECT", "0")
# conv epilogues (bias + ReLU, bias + residuals) fused after the MIOpen convolutions; "0" = A/B off
_DPT_EPI = os.environ.get("TSPLAT_DPT_EPI", "1") != "0"
# Opt-in "1": the reassemble branches of ViT layers 1-3 forked onto a side stream while the later
# blocks run (needs streams.enabled). Measured SLOWER end to end (profiles/r3/ab_r3c: C2 332 vs
# 356 views/s, C3 849 vs 887): the branches' MIOpen convolutions take CUs from the critical path
# (DINOv2 blocks and the backbone beside them) rather than filling idle ones. Round 6 (hand-written
# DINOv2 GEMMs): still slower, 444.7 vs 487.6 views/s same box (profiles/r6/ab_c2_dpt_hoist.txt).
_DPT_HOIST = os.environ.get("TSPLAT_DPT_HOIST", "0") == "1"
# bf16x3 dense mode (kernels.dense_precision): the head runs on NCHW maps instead, so its 3x3
# convolutions take the bf16x3 Winograd kernel with the ResidualConvUnit glue fused (ReLU on load,
# bias, + x, + the fusion block's skip: two launches per unit) and the 1x1s the direct kernel;
# "0" = the channels-last MIOpen chain in that mode too (A/B knob).
_DPT_NCHW3 = os.environ.get("TSPLAT_DPT_NCHW3", "1") != "0"


def _nchw3() -> bool:
    return _DPT_NCHW3 and kernels.split_mode()


def _resize(x, modifier: dict, align_corners: bool):
    """F.interpolate(x, **modifier, mode="bilinear", align_corners=...); the channels-last fp32 maps
    of the head go through one kernel (kernels.resize_bilinear_nhwc) instead of torch's NHWC
    interpolation kernel."""
    # (bilinear upsampling runs in fp32 under autocast: a bf16 map is widened first, as autocast
    # itself would, and then takes the kernel instead of torch's NHWC kernel, 88 us per call at C3)
    if (_DPT_EPI and align_corners and x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 4 == 0
            and torch.is_autocast_enabled("cuda") and x.is_contiguous(memory_format=torch.channels_last)):
        x = x.float().contiguous(memory_format=torch.channels_last)
    if (_DPT_EPI and align_corners and x.is_cuda and x.dtype == torch.float32 and x.shape[1] % 4 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        if "size" in modifier:
            size = modifier["size"]
        else:
            sf = modifier["scale_factor"]
            size = (int(x.shape[-2] * sf), int(x.shape[-1] * sf))
        return kernels.resize_bilinear_nhwc(x, size)
    if _DPT_EPI and align_corners and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.is_contiguous():
        # NCHW fp32 (the head's final resize; every config, fp32 included -- test_depth_anything_gpu
        # covers it in fp32): PyTorch's generic NCHW kernel took 0.87 ms per call at C3's batch 8
        if "size" in modifier:
            size = modifier["size"]
        else:
            sf = modifier["scale_factor"]
            size = (int(x.shape[-2] * sf), int(x.shape[-1] * sf))
        return kernels.interpolate_bilinear_ac(x, size)
    return F.interpolate(x, **modifier, mode="bilinear", align_corners=align_corners)


class ResidualConvUnit(nn.Module):
    def __init__(self, features, activation, bn):
        super().__init__()
        self.bn = bn
        self.conv1 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)
        self.conv2 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)
        if bn:
            self.bn1 = nn.BatchNorm2d(features)
            self.bn2 = nn.BatchNorm2d(features)
        self.activation = activation

    def _epilogue_ok(self, x) -> bool:
        return (_DPT_EPI and not self.bn and isinstance(self.activation, nn.ReLU) and x.dtype == torch.float32
                and self.conv1.weight.dtype == torch.float32 and x.shape[1] % 4 == 0
                and not torch.is_autocast_enabled("cuda"))

    def forward(self, x, skip=None):
        """out(x) + x (+ skip: the FeatureFusionBlock's other input, added in the same pass)."""
        if (_nchw3() and not self.bn and isinstance(self.activation, nn.ReLU) and x.is_cuda and x.is_contiguous()
                and kernels.conv3x3_wino_ok(x, self.conv1.weight, vs_miopen=True)
                and (skip is None or skip.is_contiguous())):
            # bf16x3 mode, NCHW: relu -> conv1 + bias, relu -> conv2 + bias + x (+ skip), two launches
            out = kernels.conv3x3_wino(x, self.conv1.weight, self.conv1.bias, relu_in=True)
            return kernels.conv3x3_wino(out, self.conv2.weight, self.conv2.bias, relu_in=True, residual=x,
                                        residual2=skip)
        if _DPT_DIRECT == "0" and self._epilogue_ok(x):
            # bias-free MIOpen convs with bias + ReLU / bias + residual(s) fused after each:
            # 3 glue launches per unit instead of 5 (6 with the fusion block's add)
            out = kernels.conv_nhwc_epilogue(self.conv1, self.activation(x), "relu")
            return kernels.conv_nhwc_epilogue(self.conv2, out, "none", x, skip)
        if (_DPT_DIRECT != "0" and not self.bn and isinstance(self.activation, nn.ReLU)
                and kernels.conv2d_nhwc_ok(x, self.conv1.weight)):
            # latency-bound levels (<= 36^2): ReLU-on-load, bias and the residual fused into the
            # channels-last direct convolution, two launches for the unit
            out = kernels.conv2d_nhwc(x, self.conv1.weight, self.conv1.bias, relu_in=True)
            y = kernels.conv2d_nhwc(out, self.conv2.weight, self.conv2.bias, residual=x, relu_in=True)
            return y if skip is None else skip + y
        out = self.conv1(self.activation(x))
        if self.bn:
            out = self.bn1(out)
        out = self.conv2(self.activation(out))
        if self.bn:
            out = self.bn2(out)
        return out + x if skip is None else skip + (out + x)


class FeatureFusionBlock(nn.Module):
    def __init__(self, features, activation, bn=False, align_corners=True, size=None):
        super().__init__()
        self.align_corners = align_corners
        self.out_conv = nn.Conv2d(features, features, kernel_size=1, stride=1, padding=0, bias=True)
        self.resConfUnit1 = ResidualConvUnit(features, activation, bn)
        self.resConfUnit2 = ResidualConvUnit(features, activation, bn)
        self.size = size

    def forward(self, *xs, size=None):
        output = xs[0]
        if len(xs) == 2:
            output = self.resConfUnit1(xs[1], skip=output)  # xs[0] + unit(xs[1])
        output = self.resConfUnit2(output)
        if size is None and self.size is None:
            modifier = {"scale_factor": 2}
        elif size is None:
            modifier = {"size": self.size}
        else:
            modifier = {"size": size}
        output = _resize(output, modifier, self.align_corners)
        if _DPT_DIRECT == "1" and kernels.conv2d_nhwc_ok(output, self.out_conv.weight):
            return kernels.conv2d_nhwc(output, self.out_conv.weight, self.out_conv.bias)
        return self.out_conv(output)


class _Scratch(nn.Module):
    pass


class DPTHead(nn.Module):
    def __init__(self, in_channels, features=256, use_bn=False, out_channels=(256, 512, 1024, 1024),
                 use_clstoken=False):
        super().__init__()
        if use_clstoken:
            raise NotImplementedError("Depth-Anything-V2 ViT-B runs without the class-token readout")
        self.use_clstoken = use_clstoken
        self.projects = nn.ModuleList([nn.Conv2d(in_channels, oc, kernel_size=1, stride=1, padding=0)
                                       for oc in out_channels])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(out_channels[0], out_channels[0], kernel_size=4, stride=4, padding=0),
            nn.ConvTranspose2d(out_channels[1], out_channels[1], kernel_size=2, stride=2, padding=0),
            nn.Identity(),
            nn.Conv2d(out_channels[3], out_channels[3], kernel_size=3, stride=2, padding=1)])
        s = _Scratch()
        s.layer1_rn = nn.Conv2d(out_channels[0], features, 3, 1, 1, bias=False)
        s.layer2_rn = nn.Conv2d(out_channels[1], features, 3, 1, 1, bias=False)
        s.layer3_rn = nn.Conv2d(out_channels[2], features, 3, 1, 1, bias=False)
        s.layer4_rn = nn.Conv2d(out_channels[3], features, 3, 1, 1, bias=False)
        s.stem_transpose = None
        act = nn.ReLU(False)
        s.refinenet1 = FeatureFusionBlock(features, act, bn=use_bn)
        s.refinenet2 = FeatureFusionBlock(features, act, bn=use_bn)
        s.refinenet3 = FeatureFusionBlock(features, act, bn=use_bn)
        s.refinenet4 = FeatureFusionBlock(features, act, bn=use_bn)
        s.output_conv1 = nn.Conv2d(features, features // 2, kernel_size=3, stride=1, padding=1)
        s.output_conv2 = nn.Sequential(
            nn.Conv2d(features // 2, 32, kernel_size=3, stride=1, padding=1), nn.ReLU(True),
            nn.Conv2d(32, 1, kernel_size=1, stride=1, padding=0), nn.ReLU(True), nn.Identity())
        self.scratch = s

    def _channels_last_weights(self):
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)) and m.weight.dim() == 4:
                m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
        self._cl_done = True

    def prepare(self, is_cuda: bool):
        if _DPT_CL_WEIGHTS and not getattr(self, "_cl_done", False) and is_cuda and not _nchw3():
            self._channels_last_weights()

    def reassemble(self, i, x, patch_h, patch_w):
        """Branch i of the head up to layer{i+1}_rn (reference dpt.py:121-140): tokens [B, N, C] ->
        project (1x1) -> resize (convT / identity / strided conv) -> 3x3 layer_rn."""
        x = x.permute(0, 2, 1).reshape((x.shape[0], x.shape[-1], patch_h, patch_w))
        if _nchw3():  # NCHW maps for the bf16x3 kernels (the permuted view is channels-last)
            x = self.resize_layers[i](self.projects[i](x.contiguous())).contiguous()
            return getattr(self.scratch, f"layer{i + 1}_rn")(x).contiguous()
        x = self.resize_layers[i](self.projects[i](x))
        return getattr(self.scratch, f"layer{i + 1}_rn")(x)

    def forward(self, out_features, patch_h, patch_w, rn=None):
        """`rn` (not in the reference): branch outputs already computed by `reassemble` (None
        entries are computed here)."""
        self.prepare(out_features[0][0].is_cuda)
        rn = list(rn) if rn is not None else [None] * len(out_features)
        for i, x in enumerate(out_features):
            if rn[i] is None:
                rn[i] = self.reassemble(i, x[0], patch_h, patch_w)
        layer_1_rn, layer_2_rn, layer_3_rn, layer_4_rn = rn
        s = self.scratch
        path_4 = s.refinenet4(layer_4_rn, size=layer_3_rn.shape[2:])
        path_3 = s.refinenet3(path_4, layer_3_rn, size=layer_2_rn.shape[2:])
        path_2 = s.refinenet2(path_3, layer_2_rn, size=layer_1_rn.shape[2:])
        path_1 = s.refinenet1(path_2, layer_1_rn)
        final_out = s.output_conv1(path_1)
        out_feature = final_out.clone().detach()
        final_out = _resize(final_out, {"size": (int(patch_h * 14), int(patch_w * 14))}, True)
        oc = s.output_conv2
        if _nchw3() and final_out.is_contiguous() and kernels.conv3x3_wino_ok(final_out, oc[0].weight, vs_miopen=True):
            h = kernels.conv3x3_wino(final_out, oc[0].weight, oc[0].bias, act="relu")
            return oc[4](oc[3](oc[2](h))), out_feature
        if (_DPT_EPI and final_out.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")
                and final_out.is_cuda and final_out.is_contiguous(memory_format=torch.channels_last)):
            # conv -> ReLU as conv + (bias, ReLU) epilogue; the 1-channel tail stays on the modules
            h = kernels.conv_nhwc_epilogue(oc[0], final_out, "relu")
            return oc[4](oc[3](oc[2](h))), out_feature
        return oc(final_out), out_feature


class DepthAnythingV2(nn.Module):
    def __init__(self, encoder="vitl", features=256, out_channels=(256, 512, 1024, 1024), use_bn=False,
                 use_clstoken=False):
        super().__init__()
        self.intermediate_layer_idx = {"vits": [2, 5, 8, 11], "vitb": [2, 5, 8, 11], "vitl": [4, 11, 17, 23]}
        self.encoder = encoder
        self.pretrained = DINOv2(model_name=encoder)
        self.depth_head = DPTHead(self.pretrained.embed_dim, features, use_bn, out_channels=out_channels,
                                  use_clstoken=use_clstoken)

    def forward(self, x):
        patch_h, patch_w = x.shape[-2] // 14, x.shape[-1] // 14
        head = self.depth_head
        head.prepare(x.is_cuda)
        n_take = len(self.intermediate_layer_idx[self.encoder])
        pending = {}

        def on_output(k, tokens):
            # branches 1-3 start on a side stream as soon as their ViT layer exists and overlap the
            # remaining blocks; the last one has nothing left to overlap and runs inline
            if k + 1 < n_take and _DPT_HOIST and streams.enabled(tokens.device):
                pending[k] = streams.fork(tokens.device, head.reassemble, k, tokens[:, 1:], patch_h, patch_w,
                                          slot=1)

        from ...misc.benchmarker import stage

        with stage(None, "da_dinov2"):  # diagnostic sub-stage marks (TSPLAT_MARKS / TSPLAT_ROCTX)
            features = self.pretrained.get_intermediate_layers(x, self.intermediate_layer_idx[self.encoder],
                                                               return_class_token=True, on_output=on_output)
        rn = [streams.join(pending[k]) if k in pending else None for k in range(n_take)]
        with stage(None, "da_dpt"):
            depth, out_features = head(features, patch_h, patch_w, rn=rn)
        return F.relu(depth).squeeze(1), out_features
