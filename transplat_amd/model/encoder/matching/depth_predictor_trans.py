"""Cost-volume depth predictor (reference src/model/encoder/matching/depth_predictor_trans.py).

IMPORTANT (as in the reference): tensors here are (v b)-ordered, not (b v).
Stages: camera prep -> coarse + fine UV correlation (gfx950 kernels, grid
computed in-kernel) -> cost-volume U-Net -> softmax depth -> refine U-Net -> Gaussian heads.
Parameter names match the reference for checkpoint loading.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from einops import rearrange, repeat
from torch import nn

from .... import kernels, streams
from ....misc.benchmarker import stage
from ...utils.cam_param_encoder import cam_param_encoder
from ...utils.uv_transformer import UVTransformer
from .ldm_unet import UNetModel, run_sequential


def _conv_upsample_gelu(seq: nn.Sequential, x):
    """Sequential(Conv2d, Upsample(bilinear, align_corners=True), GELU): the bias-free convolution,
    then interpolation + bias + GELU in one pass over the full-resolution map
    (kernels.upsample_bilinear_act) instead of bias add, interpolation and GELU kernels."""
    conv, up, act = seq
    # (under bf16 autocast the convolution runs in bf16 and the interpolation + GELU in fp32, which
    # is what autocast does with this Sequential: upsample_bilinear2d is on its fp32 list)
    if (not isinstance(act, nn.GELU) or act.approximate != "none" or up.mode != "bilinear"
            or not up.align_corners or float(up.scale_factor) != int(up.scale_factor)):
        return seq(x)
    if kernels.conv3x3_wino_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, vs_miopen=True):
        y = kernels.conv3x3_wino(x, conv.weight, None)  # (MIOpen 53 us at 256 -> 128 / 64^2; bf16x3 ~24 us)
    else:
        y = kernels.conv2d_fallback(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    return kernels.upsample_bilinear_act(y, int(up.scale_factor), conv.bias, "gelu")


def _conv_gelu_conv(seq: nn.Sequential, x, extra=()):
    """Sequential(Conv2d, GELU, Conv2d) head on cat([x, *extra], 1) with each conv's bias (and the
    GELU) applied in one pass after the bias-free convolution (kernels.conv_bias_act; on the
    Winograd path the concatenation is read in place and bias / GELU are its epilogue)."""
    if not (len(seq) == 3 and isinstance(seq[1], nn.GELU) and seq[1].approximate == "none"):
        return seq(torch.cat([x, *extra], dim=1) if extra else x)
    return kernels.conv_bias_act(seq[2], kernels.conv_bias_act(seq[0], x, "gelu", site="head", extra=extra),
                                 site="head")


@torch.autocast("cuda", enabled=False)
def camera_lists(intrinsics, extrinsics, near, far, num_samples: int, h: int, w: int):
    """The camera half of prepare_feat_proj_data_lists (reference :59-109): pixel intrinsics, relative
    poses and disparity candidates 1/far + linspace(0, 1, D) (1/near - 1/far), all in (v b) order,
    fp32. Depends on the cameras only, so the encoder computes it at the start of the step on a
    side stream (EncoderTrans.forward), off the depth predictor's critical path."""
    b, v = intrinsics.shape[:2]
    pose_curr_lists = []
    init_view_order = list(range(v))
    if v > 2:
        for idx in range(1, v):
            cur_view_order = init_view_order[idx:] + init_view_order[:idx]
            cur = [kernels.small_inverse(extrinsics[:, v1].clone().detach()) @ extrinsics[:, v0].clone().detach()
                   for v0, v1 in zip(init_view_order, cur_view_order)]
            pose_curr_lists.append(torch.cat(cur, dim=0))
    else:
        pose_ref = extrinsics[:, 0].clone().detach()
        pose_tgt = extrinsics[:, 1].clone().detach()
        pose = kernels.small_inverse(pose_tgt) @ pose_ref
        pose_curr_lists = [torch.cat((pose, kernels.small_inverse(pose)), dim=0)]
    intr_curr = intrinsics[:, :, :3, :3].clone().detach()
    intr_curr[:, :, 0, :] *= float(w)
    intr_curr[:, :, 1, :] *= float(h)
    intr_curr = rearrange(intr_curr, "b v ... -> (v b) ...", b=b, v=v)
    min_depth = rearrange(1.0 / far.clone().detach(), "b v -> (v b) 1")
    max_depth = rearrange(1.0 / near.clone().detach(), "b v -> (v b) 1")
    depth_candi_curr = (min_depth + torch.linspace(0.0, 1.0, num_samples, device=min_depth.device).unsqueeze(0)
                        * (max_depth - min_depth)).float()
    depth_candi_curr = repeat(depth_candi_curr, "vb d -> vb d () ()")
    return intr_curr, pose_curr_lists, depth_candi_curr


def match_img2world(intr_curr, extrinsics):
    """[(v b), 16] c2w @ inv(K_pixel) of every view (reference :241-248), the camera-parameter
    encoder's input in match_two."""
    b, v = extrinsics.shape[:2]
    with torch.autocast("cuda", enabled=False):
        camk = torch.eye(4, device=intr_curr.device).view(1, 4, 4).repeat(intr_curr.shape[0], 1, 1).float()
        camk[:, :3, :3] = intr_curr
        c2w = rearrange(extrinsics.clone().detach(), "b v ... -> (v b) ...", b=b, v=v)
        return torch.matmul(c2w, kernels.small_inverse(camk)).reshape(-1, 16)


def prepare_feat_proj_data_lists(features, intrinsics, extrinsics, near, far, num_samples, cams=None):
    """(reference :59-109) per-view features, pixel intrinsics, relative poses and disparity
    candidates 1/far + linspace(0, 1, D) (1/near - 1/far), all in (v b) order. Camera math stays
    fp32 when the dense layers run under bf16 autocast. cams: camera_lists' result, if already
    computed."""
    b, v, _, h, w = features.shape
    feat_lists = [rearrange(features, "b v ... -> (v b) ...")]
    for idx in range(1, v):
        # features[:, cur_view_order] as a roll (list indexing is a host copy: not graph-capturable)
        feat_lists.append(rearrange(torch.roll(features, -idx, dims=1), "b v ... -> (v b) ..."))
    if cams is None:
        cams = camera_lists(intrinsics, extrinsics, near, far, num_samples, h, w)
    intr_curr, pose_curr_lists, depth_candi_curr = cams
    return feat_lists, intr_curr, pose_curr_lists, depth_candi_curr.type_as(features)


# view pairs matched for V > 2 in the reference's order (depth_predictor_trans.py:351-414): the ring
# (i, i+1) first, then for V = 4 the diagonals (0, 2), (1, 3)
_VIEW_PAIRS = {3: ((0, 1), (1, 2), (2, 0)), 4: ((0, 1), (1, 2), (2, 3), (3, 0), (0, 2), (1, 3))}


class DepthPredictorTrans(nn.Module):
    def __init__(self, feature_channels=128, upscale_factor=4, num_depth_candidates=32, costvolume_unet_feat_dim=128,
                 costvolume_unet_channel_mult=(1, 1, 1), costvolume_unet_attn_res=(), gaussian_raw_channels=-1,
                 gaussians_per_pixel=1, num_views=2, depth_unet_feat_dim=64, depth_unet_attn_res=(),
                 depth_unet_channel_mult=(1, 1, 1), DA_size=128, **kwargs):
        super().__init__()
        self.num_depth_candidates = num_depth_candidates
        self.regressor_feat_dim = costvolume_unet_feat_dim
        self.upscale_factor = upscale_factor
        input_channels = num_depth_candidates + feature_channels
        channels = self.regressor_feat_dim
        self.corr_refine_net = nn.Sequential(
            nn.Conv2d(input_channels, channels, 3, 1, 1), nn.GroupNorm(8, channels), nn.GELU(),
            UNetModel(image_size=None, in_channels=channels, model_channels=channels, out_channels=channels,
                      num_res_blocks=1, attention_resolutions=costvolume_unet_attn_res,
                      channel_mult=costvolume_unet_channel_mult, num_head_channels=32, dims=2, postnorm=True,
                      num_frames=num_views, use_cross_view_self_attn=True),
            nn.Conv2d(channels, num_depth_candidates, 3, 1, 1))
        self.regressor_residual = nn.Conv2d(input_channels, num_depth_candidates, 1, 1, 0)
        self.depth_head_lowres = nn.Sequential(
            nn.Conv2d(num_depth_candidates, num_depth_candidates * 2, 3, 1, 1), nn.GELU(),
            nn.Conv2d(num_depth_candidates * 2, num_depth_candidates, 3, 1, 1))
        proj_in_channels = feature_channels + feature_channels
        upsample_out_channels = feature_channels
        self.upsampler = nn.Sequential(
            nn.Conv2d(proj_in_channels, upsample_out_channels, 3, 1, 1),
            nn.Upsample(scale_factor=upscale_factor, mode="bilinear", align_corners=True), nn.GELU())
        self.proj_feature = nn.Conv2d(upsample_out_channels, depth_unet_feat_dim, 3, 1, 1)
        input_channels = 3 + 1 + depth_unet_feat_dim + 1 + 1
        channels = depth_unet_feat_dim
        self.refine_unet = nn.Sequential(
            nn.Conv2d(input_channels, channels, 3, 1, 1), nn.GroupNorm(4, channels), nn.GELU(),
            UNetModel(image_size=None, in_channels=channels, model_channels=channels, out_channels=channels,
                      num_res_blocks=1, attention_resolutions=depth_unet_attn_res,
                      channel_mult=depth_unet_channel_mult, num_head_channels=32, dims=2, postnorm=True,
                      num_frames=num_views, use_cross_view_self_attn=True))
        gau_in = depth_unet_feat_dim + 3 + feature_channels
        self.to_gaussians = nn.Sequential(
            nn.Conv2d(gau_in, gaussian_raw_channels * 2, 3, 1, 1), nn.GELU(),
            nn.Conv2d(gaussian_raw_channels * 2, gaussian_raw_channels, 3, 1, 1))
        channels = depth_unet_feat_dim
        self.to_disparity = nn.Sequential(
            nn.Conv2d(channels, channels * 2, 3, 1, 1), nn.GELU(),
            nn.Conv2d(channels * 2, gaussians_per_pixel * 2, 3, 1, 1))
        self.embed_dims = 128
        self.coarse_transformer = UVTransformer(embed_dims=self.embed_dims, mode="coarse", num_layers=1)
        self.fine_transformer = UVTransformer(embed_dims=self.embed_dims, mode="fine", num_layers=2)
        self.cam_param_encoder = cam_param_encoder(in_channels=DA_size, mid_channels=128, embed_dims=128)

    def camera_prep(self, intrinsics, extrinsics, near, far, h: int, w: int) -> dict:
        """Everything the depth predictor derives from the cameras alone (camera_lists, and
        match_two's img2world for two views), for forward(cams=...)."""
        intr, poses, disp = camera_lists(intrinsics, extrinsics, near, far, self.num_depth_candidates, h, w)
        out = {"lists": (intr, poses, disp)}
        if intrinsics.shape[1] == 2:
            out["img2world"] = match_img2world(intr, extrinsics)
        return out

    def coarse_two(self, intr_curr, pose_curr, disp_candi_curr, features):
        """(reference :236-290, first half) the coarse correlation layer of a pair of views: reads
        only the backbone features and the cameras, so the encoder runs it before Depth-Anything's
        features exist (the reference computes the camera-parameter embedding first; the two are
        independent)."""
        b, v, c, h, w = features.shape
        cameras = (intr_curr, pose_curr, disp_candi_curr.flatten(1).float())
        feat_cl = features.flatten(3).transpose(2, 3).contiguous()  # [b, v, HW, C]
        query = torch.zeros((b * v, h * w, self.embed_dims), device=features.device, dtype=features.dtype)
        corr = self.coarse_transformer([features], query, w, h, cameras=cameras, channel_last=feat_cl)
        return corr, cameras, feat_cl

    def fine_two(self, coarse, intr_curr, extrinsics, dino_feature, features, img2world=None):
        """(reference :236-290, second half) the fine layers on the coarse correlation, with the
        Depth-Anything-feature position embedding -> [(v b), D, h, w]."""
        b, v, c, h, w = features.shape
        corr, cameras, feat_cl = coarse
        if img2world is None:
            img2world = match_img2world(intr_curr, extrinsics)
        pos_feature = self.cam_param_encoder(dino_feature, img2world)  # [(v b), C, h, w]
        # (b v)-ordered channel-last query positions: the reference's bev_pos after its permutes
        bev_pos = rearrange(pos_feature, "(v b) c h w -> (b v) (h w) c", v=v, b=b).contiguous()  # read by 2 layers
        corr = self.fine_transformer([features], corr, w, h, bev_pos=bev_pos, cameras=cameras, channel_last=feat_cl)
        return rearrange(corr, "(b v) (h w) c -> (v b) c h w", b=b, v=v, h=h, w=w)

    def match_two(self, intr_curr, pose_curr, extrinsics, disp_candi_curr, dino_feature, features, img2world=None):
        """(reference :236-290) coarse then fine correlation for a pair of views -> [(v b), D, h, w]."""
        coarse = self.coarse_two(intr_curr, pose_curr, disp_candi_curr, features)
        return self.fine_two(coarse, intr_curr, extrinsics, dino_feature, features, img2world)

    def match_pairs(self, intr_curr, pose_curr_lists, extrinsics, disp_candi_curr, dino_feature, features):
        """(reference :351-414) V = 3 / 4: match_two on every pair of _VIEW_PAIRS[V], then each view's
        correlation is the mean of its halves over the pairs that contain it, taken in the
        reference's order (pairs where it comes first, then pairs where it comes second).
        pose_curr_lists[k] holds inv(E[(a + k + 1) % V]) E[a] for view a, so pair (a, c) uses
        lists[(c - a - 1) % V][a] and lists[(a - c - 1) % V][c]. Generalised to batch b > 1 by
        taking (v b) blocks (the reference indexes single rows, i.e. assumes b = 1)."""
        b, v = features.shape[:2]
        blk = lambda t, a: t[a * b:(a + 1) * b]
        parts = []
        for a, c in _VIEW_PAIRS[v]:
            pose = torch.cat((blk(pose_curr_lists[(c - a - 1) % v], a), blk(pose_curr_lists[(a - c - 1) % v], c)))
            pair = lambda t: torch.cat((blk(t, a), blk(t, c)))
            corr = self.match_two(pair(intr_curr), pose, torch.stack((extrinsics[:, a], extrinsics[:, c]), 1),
                                  pair(disp_candi_curr), pair(dino_feature),
                                  torch.stack((features[:, a], features[:, c]), 1))
            parts.append((corr[:b], corr[b:]))
        per_view = []
        for k in range(v):
            halves = [p[0] for (a, _), p in zip(_VIEW_PAIRS[v], parts) if a == k]
            halves += [p[1] for (_, c), p in zip(_VIEW_PAIRS[v], parts) if c == k]
            per_view.append(torch.stack(halves, dim=0).mean(dim=0))
        return torch.cat(per_view, dim=0)  # (v b)

    def _projection(self, feat01, cnn_features):  # (reference :448-452) reads backbone features only
        proj_feat_in_fullres = _conv_upsample_gelu(self.upsampler, torch.cat((feat01, cnn_features), dim=1))
        return proj_feat_in_fullres, self.proj_feature(proj_feat_in_fullres)

    def begin(self, features, intrinsics, extrinsics, near, far, cnn_features=None, benchmarker=None, cams=None,
              fork_projection=True):
        """The part of forward that reads only the backbone's outputs and the cameras -- 4a's feature
        lists, the full-resolution projection (forked beside the cost volume) and, for two views,
        the coarse correlation layer -- so that the encoder can run it on the backbone's branch while
        Depth-Anything is still computing; forward(begun=...) continues from it. fork_projection=False
        (inside a forked branch, which must not fork again under capture): forward forks it."""
        b, v, c, h, w = features.shape

        # the reference's stage tags (depth_predictor_trans.py:320-456) as roctx ranges
        with stage(benchmarker, "encoder_4a_prep_features"):
            if cnn_features is not None:
                cnn_features = rearrange(cnn_features, "b v ... -> (v b) ...")
            feat_comb_lists, intr_curr, pose_curr_lists, disp_candi_curr = prepare_feat_proj_data_lists(
                features, intrinsics, extrinsics, near, far, num_samples=self.num_depth_candidates,
                cams=cams["lists"] if cams is not None else None)
            feat01 = feat_comb_lists[0]
            # the full-resolution feature projection runs on a side stream beside the cost volume
            # (matching, refine U-Net, depth head: a chain of 64^2 launches), transplat_amd/streams.py
            proj = (streams.fork(features.device, self._projection, feat01, cnn_features) if fork_projection
                    else (feat01, cnn_features))
        coarse = None
        if v == 2:
            with stage(None, "dp_coarse"):  # diagnostic sub-stage mark
                coarse = self.coarse_two(intr_curr, pose_curr_lists[0], disp_candi_curr, features)
        return {"lists": (intr_curr, pose_curr_lists, disp_candi_curr), "feat01": feat01, "proj": proj,
                "proj_forked": fork_projection, "coarse": coarse}

    def forward(self, features, intrinsics, extrinsics, near, far, gaussians_per_pixel=1, deterministic=True,
                extra_info=None, cnn_features=None, da_depth=None, dino_feature=None, benchmarker=None, cams=None,
                begun=None):
        b, v, c, h, w = features.shape
        if begun is None:
            begun = self.begin(features, intrinsics, extrinsics, near, far, cnn_features, benchmarker, cams)
        intr_curr, pose_curr_lists, disp_candi_curr = begun["lists"]
        feat01, proj = begun["feat01"], begun["proj"]
        if not begun["proj_forked"]:
            proj = streams.fork(features.device, self._projection, *proj)
        if da_depth is not None:
            da_depth = rearrange(da_depth, "b v ... -> (v b) ...")
        if dino_feature is not None:
            dino_feature = rearrange(dino_feature, "b v ... -> (v b) ...")
            dino_feature = kernels.interpolate_bilinear_ac(dino_feature, (h, w))
        with stage(benchmarker, "encoder_4b_cost_volume_matching"):
            img2world = cams.get("img2world") if cams is not None else None
            if begun["coarse"] is not None:
                raw_correlation_in = torch.cat((self.fine_two(begun["coarse"], intr_curr, extrinsics, dino_feature,
                                                              features, img2world), feat01), dim=1)
            else:
                raw_correlation_in = self._match(v, intr_curr, pose_curr_lists, extrinsics, disp_candi_curr,
                                                 dino_feature, features, feat01, img2world)
        with stage(benchmarker, "encoder_4c_cost_volume_unet"):
            raw_correlation = (run_sequential(self.corr_refine_net, raw_correlation_in)
                               + self.regressor_residual(raw_correlation_in))
        with stage(benchmarker, "encoder_4d_coarse_depth"):
            coarse_disps, pdf_max, fullres_disps = self._coarse_depth(raw_correlation, disp_candi_curr)
        with stage(benchmarker, "encoder_4e_depth_refine_unet"):
            proj_feat_in_fullres, proj_feature = streams.join(proj)
            refine_out = run_sequential(self.refine_unet, torch.cat(
                (extra_info["images"], da_depth, proj_feature, fullres_disps, pdf_max), dim=1))
        with stage(benchmarker, "encoder_4f_gaussian_head"):
            raw_gaussians = _conv_gelu_conv(self.to_gaussians, refine_out,
                                            extra=(extra_info["images"], proj_feat_in_fullres))
            raw_gaussians = rearrange(raw_gaussians, "(v b) c h w -> b v (h w) c", v=v, b=b)
            head = _conv_gelu_conv(self.to_disparity, refine_out)
            if gaussians_per_pixel == 1:  # the tail below as one kernel, written in the (b v) layouts
                depths, densities = kernels.depth_tail(fullres_disps, head, near, far)
                depths = depths.view(b, v, -1, 1, 1)
                densities = densities.view(b, v, -1, 1, 1)
            else:
                delta_disps, raw_densities = head.split(gaussians_per_pixel, dim=1)
                densities = repeat(F.sigmoid(raw_densities), "(v b) dpt h w -> b v (h w) srf dpt", b=b, v=v, srf=1)
                fine_disps = (fullres_disps + delta_disps).clamp(1.0 / rearrange(far, "b v -> (v b) () () ()"),
                                                                 1.0 / rearrange(near, "b v -> (v b) () () ()"))
                depths = repeat(1.0 / fine_disps, "(v b) dpt h w -> b v (h w) srf dpt", b=b, v=v, srf=1)
        return depths, densities, raw_gaussians

    def _match(self, v, intr_curr, pose_curr_lists, extrinsics, disp_candi_curr, dino_feature, features, feat01,
               img2world=None):
        if v == 2:
            raw_correlation_in = self.match_two(intr_curr, pose_curr_lists[0], extrinsics, disp_candi_curr,
                                                dino_feature, features, img2world)
        elif v in _VIEW_PAIRS:
            raw_correlation_in = self.match_pairs(intr_curr, pose_curr_lists, extrinsics, disp_candi_curr,
                                                  dino_feature, features)
        else:
            raise NotImplementedError(f"{v} context views (the reference handles 2, 3 and 4)")
        return torch.cat((raw_correlation_in, feat01), dim=1)

    def _coarse_depth(self, raw_correlation, disp_candi_curr):
        logits = _conv_gelu_conv(self.depth_head_lowres, raw_correlation)
        if logits.dtype == torch.float32:  # softmax, expected disparity and max in one pass
            coarse_disps, pdf_max = kernels.depth_softmax(logits, disp_candi_curr)
        else:
            pdf = F.softmax(logits, dim=1)
            coarse_disps = (disp_candi_curr * pdf).sum(dim=1, keepdim=True)
            pdf_max = torch.max(pdf, dim=1, keepdim=True)[0]
        pdf_max = F.interpolate(pdf_max, scale_factor=self.upscale_factor)
        up = int(self.upscale_factor)  # align_corners: the ratio comes from the sizes, as torch's
        fullres_disps = kernels.interpolate_bilinear_ac(coarse_disps, (coarse_disps.shape[-2] * up,
                                                                       coarse_disps.shape[-1] * up))
        return coarse_disps, pdf_max, fullres_disps
