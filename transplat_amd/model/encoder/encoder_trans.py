"""TranSplat encoder: context views -> per-pixel 3-D Gaussians
(reference src/model/encoder/encoder_trans.py:40-376, same constructor config and forward
signature, same module names -> `encoder.*` checkpoint keys load).

Stages (reference bench tags encoder_1..5): intrinsics prep, multi-view backbone (gfx950 window
attention), Depth-Anything-V2 (no_grad), cost-volume depth predictor (gfx950 correlation
kernels), Gaussian adapter (e3nn-free SH rotation). No host synchronisation between stages
(the reference forces torch.cuda.synchronize() around each).
"""
from __future__ import annotations

import os

from contextlib import nullcontext
from dataclasses import dataclass, field
from typing import List, Literal, Optional

import torch
import torch.nn.functional as F
from einops import rearrange
from torch import nn

from ... import kernels, streams
from ...misc.benchmarker import stage
from ..depth_anything.dpt import DepthAnythingV2
from ..types import Gaussians
from .backbone.backbone_multiview import BackboneMultiview
from .common.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg
from .encoder import Encoder
from .matching.depth_predictor_trans import DepthPredictorTrans

_DA_CONFIGS = {
    "vits": {"encoder": "vits", "features": 64, "out_channels": [48, 96, 192, 384]},
    "vitb": {"encoder": "vitb", "features": 128, "out_channels": [96, 192, 384, 768]},
    "vitl": {"encoder": "vitl", "features": 256, "out_channels": [256, 512, 1024, 1024]},
}


@dataclass
class OpacityMappingCfg:
    initial: float = 0.0
    final: float = 0.0
    warm_up: int = 1


@dataclass
class EncoderTransCfg:
    """Defaults = config/model/encoder/trans.yaml overridden by config/experiment/re10k.yaml."""

    name: Literal["trans"] = "trans"
    d_feature: int = 128
    num_depth_candidates: int = 128
    num_surfaces: int = 1
    gaussian_adapter: GaussianAdapterCfg = field(default_factory=GaussianAdapterCfg)
    opacity_mapping: OpacityMappingCfg = field(default_factory=OpacityMappingCfg)
    gaussians_per_pixel: int = 1
    unimatch_weights_path: Optional[str] = None
    downscale_factor: int = 4
    shim_patch_size: int = 4
    multiview_trans_attn_split: int = 2
    costvolume_unet_feat_dim: int = 128
    costvolume_unet_channel_mult: List[int] = field(default_factory=lambda: [1, 1, 1])
    costvolume_unet_attn_res: List[int] = field(default_factory=lambda: [4])
    depth_unet_feat_dim: int = 32
    depth_unet_attn_res: List[int] = field(default_factory=lambda: [16])
    depth_unet_channel_mult: List[int] = field(default_factory=lambda: [1, 1, 1, 1, 1])
    wo_depth_refine: bool = False
    wo_cost_volume: bool = False
    wo_cost_volume_refine: bool = False
    num_context_views: int = 2  # the reference reads it from the global dataset config
    da_encoder: str = "vitb"
    # Arithmetic of the conv / GEMM layers around the hand-written kernels (CNN, cam encoders,
    # DA-V2, U-Nets, heads): "fp32" (exact fp32, parity mode), "bf16x3" (split-bf16 products with
    # fp32 accumulation -- the stand-in for the reference's TF32, src/main.py:15, more precise than
    # it; kernels.dense_precision) or "bf16" (autocast). The rasterizer and the correlation gathers
    # always run fp32; the fine-cross correlation TABLE is a dense GEMM and follows dense_dtype
    # (bf16x3: one split-bf16 hipBLASLt GEMM over K' = 3K, kernels.uv_cross).
    dense_dtype: str = "fp32"
    # Window attention (T2): "auto" (bf16 MFMA under bf16 dense layers, bf16x3 under bf16x3 ones,
    # else exact fp32; kernels.auto_attention), "fp32", "bf16x3" or "bf16" (config C3 as
    # BASELINE.json states it: bf16 attention beside fp32-class dense layers).
    attn_dtype: str = "auto"


# camera-only prep of the depth predictor and the adapter on the backbone's branch
# (TSPLAT_CAM_HOIST=0: computed where it is used, the A/B knob)
_CAM_HOIST = os.environ.get("TSPLAT_CAM_HOIST", "1") == "1"
# the depth predictor's backbone-only first part on the backbone's branch ("1"; default "0": after the
# join). Round 6: with it on the branch, hipGraph replays of the step were not the eager step (the
# encoder's Gaussians moved in 4-8 of 12 replays, means by up to 17; tools/enc_graph_race.py,
# profiles/r6/graph_race.log), with it after the join 0 of 32. The coarse correlation kernel itself
# is deterministic beside a busy stream and in two-stream graphs, and reads nothing outside its
# inputs (tools/coarse_stress.py, tools/coarse_oob.py); the hazard is in the branch arrangement,
# whose cause was not pinned down. Cost: C2 ~1 % (486.6 vs 490.9 views/s same box).
_DP_BEGIN_SIDE = os.environ.get("TSPLAT_DP_BEGIN_SIDE", "0") == "1"
# Depth-Anything on the side stream and the backbone on the current one (A/B; with TSPLAT_SIDE_PRIO)
_DA_SIDE = os.environ.get("TSPLAT_DA_SIDE", "0") == "1"


class EncoderTrans(Encoder[EncoderTransCfg]):
    def __init__(self, cfg: EncoderTransCfg) -> None:
        super().__init__(cfg)
        self.backbone = BackboneMultiview(feature_channels=cfg.d_feature, downscale_factor=cfg.downscale_factor)
        self.gaussian_adapter = GaussianAdapter(cfg.gaussian_adapter)
        da = _DA_CONFIGS[cfg.da_encoder]
        self.da_model = DepthAnythingV2(**da).eval()
        for p in self.da_model.parameters():
            p.requires_grad = False
        self.depth_predictor = DepthPredictorTrans(
            feature_channels=cfg.d_feature, upscale_factor=cfg.downscale_factor,
            num_depth_candidates=cfg.num_depth_candidates, costvolume_unet_feat_dim=cfg.costvolume_unet_feat_dim,
            costvolume_unet_channel_mult=tuple(cfg.costvolume_unet_channel_mult),
            costvolume_unet_attn_res=tuple(cfg.costvolume_unet_attn_res),
            gaussian_raw_channels=cfg.num_surfaces * (self.gaussian_adapter.d_in + 2),
            gaussians_per_pixel=cfg.gaussians_per_pixel, num_views=cfg.num_context_views,
            depth_unet_feat_dim=cfg.depth_unet_feat_dim, depth_unet_attn_res=cfg.depth_unet_attn_res,
            depth_unet_channel_mult=cfg.depth_unet_channel_mult, DA_size=da["features"] // 2)
        # constants as non-persistent buffers: no host->device copy inside forward (graph capture)
        self.register_buffer("img_mean", torch.tensor([0.485, 0.456, 0.406]), persistent=False)
        self.register_buffer("img_std", torch.tensor([0.229, 0.224, 0.225]), persistent=False)
        # every plain Conv2d: the large 3x3s on the Winograd fp32 MFMA kernel, the rest unchanged
        # (kernels.conv2d_forward; CPU tensors and bf16 autocast keep the module's own conv)
        kernels.install_conv2d_dispatch(self)
        # every plain Linear: split-bf16 GEMMs in dense_dtype "bf16x3" (kernels.linear_forward)
        kernels.install_linear_dispatch(self)

    def map_pdf_to_opacity(self, pdf, global_step: int):
        """(reference :139-152)"""
        cfg = self.cfg.opacity_mapping
        x = cfg.initial + min(global_step / cfg.warm_up, 1) * (cfg.final - cfg.initial)
        exponent = 2**x
        return 0.5 * (1 - (1 - pdf) ** exponent + pdf ** (1 / exponent))

    def normalize_images(self, images):
        shape = [*[1] * (images.dim() - 3), 3, 1, 1]
        return (images - self.img_mean.reshape(*shape)) / self.img_std.reshape(*shape)

    def _dense(self):
        if self.cfg.dense_dtype == "bf16":
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16)
        if self.cfg.dense_dtype == "bf16x3":
            return kernels.dense_precision("bf16x3")
        if self.cfg.dense_dtype != "fp32":
            raise ValueError(f"dense_dtype {self.cfg.dense_dtype!r}")
        return nullcontext()

    def forward(self, context: dict, global_step: int = 0, deterministic: bool = False,
                visualization_dump: Optional[dict] = None, scene_names=None, benchmarker=None,
                analyze_feature_depth: bool = False, enable_saes: bool = False, saes_config=None) -> Gaussians:
        device = context["image"].device
        b, v, _, h, w = context["image"].shape

        def bench(tag):  # the reference's stage tags (encoder_trans.py:188-294) as roctx ranges
            return stage(benchmarker, tag)

        def prep_intrinsics(intrinsics, extrinsics):  # the backbone's camera input (runs on its stream)
            with bench("encoder_1_prep_intrinsics"):
                intr_curr = intrinsics[:, :, :3, :3].clone().detach()
                intr_curr[:, :, 0, :] *= float(w)
                intr_curr[:, :, 1, :] *= float(h)
                camk = torch.eye(4, device=device).view(1, 1, 4, 4).repeat(b, v, 1, 1).float()
                camk[:, :, :3, :3] = intr_curr
                return torch.matmul(extrinsics.clone().detach(), kernels.small_inverse(camk))

        def camera_consts(intrinsics, extrinsics, near, far):
            # everything the depth predictor and the adapter derive from the cameras alone: computed
            # on the backbone's branch, beside Depth-Anything, instead of as ~40 tiny launches on the
            # critical path before those stages (a stream of its own measured 2.7 % slower)
            with bench("encoder_cameras"):
                f = self.cfg.downscale_factor  # the depth predictor works on the feature maps
                dp = self.depth_predictor.camera_prep(intrinsics, extrinsics, near, far, h // f, w // f)
                ad = kernels.adapter_camera_consts(extrinsics, intrinsics, (h, w), self.gaussian_adapter.d_sh)
            return dp, ad

        def depth_anything(images):
            with bench("encoder_3_depth_anything"), torch.no_grad(), self._dense():
                # channel order (2, 0, 1) as the reference, by slicing: a list index would be a
                # pageable host-to-device copy, which is not allowed inside hipGraph capture
                da_images = self.normalize_images(images)
                da_images = torch.cat((da_images[:, :, 2:3], da_images[:, :, 0:2]), dim=2)
                da_images = da_images.reshape(b * v, 3, h, w)
                da_images = kernels.interpolate_bilinear_ac(da_images, (252, 252))
                da_depth, out_feature = self.da_model(da_images)
                da_depth = kernels.interpolate_bilinear_ac(da_depth[None].float().contiguous(), (h, w))
                da_depth = da_depth.view(b, v, 1, h, w).flatten(2)
                # per-view min / max in two aminmax stages (rows of w, then the h row results): the
                # single-row reductions ran on 2 workgroups each (~20 us apiece); exact either way
                lo, hi = torch.aminmax(da_depth.view(b, v, h, w), dim=-1)
                da_min = lo.amin(dim=-1, keepdim=True)
                da_max = hi.amax(dim=-1, keepdim=True)
                da_depth = ((da_depth - da_min) / (da_max - da_min)).reshape(b, v, 1, h, w)
                return da_depth, out_feature.float()

        attn = self.cfg.attn_dtype
        if attn == "auto":
            attn = kernels.auto_attention(self.cfg.dense_dtype)

        def backbone(images, intrinsics, extrinsics, near, far):
            img2world = prep_intrinsics(intrinsics, extrinsics)
            with bench("encoder_2_backbone"), self._dense(), kernels.attention_precision(attn):
                tf, cf = self.backbone(images, attn_splits=self.cfg.multiview_trans_attn_split,
                                       return_cnn_features=True, img2world=img2world)
            # the backbone's branch finishes well before Depth-Anything: its slack takes the camera prep
            cams = camera_consts(intrinsics, extrinsics, near, far) if _CAM_HOIST else (None, None)
            return tf.float(), cf.float(), cams

        # Stages 2 and 3 read only the context images, and the depth predictor's first part (its
        # feature lists and the coarse correlation layer) reads only the backbone's outputs and the
        # cameras: on a GPU, the backbone, the camera prep and that first part run on a side stream
        # (transplat_amd/streams.py; captured into the step's hipGraph as a parallel branch) beside
        # Depth-Anything -- together shorter than it. Both are chains of small launches (DINOv2's
        # M = 650 GEMMs, the MVT's 256-workgroup kernels) that leave CUs idle on their own.
        # Depth-Anything stays on the current stream: the other arrangement (it on the side stream,
        # the backbone here) measured 1 % slower, its DPT then losing CUs to the MVT (C2 426 vs 430
        # views/s same box, profiles/r5/ab_da_side.txt); and a fork from a side stream inside hipGraph
        # capture crashes HIP's capture_end, so the depth predictor's projection fork waits for the
        # current stream.
        def dp_begin(tf, cf, dp_cams, fork_projection):
            with bench("encoder_4_depth_predictor"), self._dense():
                return self.depth_predictor.begin(tf, context["intrinsics"], context["extrinsics"], context["near"],
                                                  context["far"], cnn_features=cf, benchmarker=benchmarker,
                                                  cams=dp_cams, fork_projection=fork_projection)

        def backbone_branch(*ctx):
            tf, cf, cams = backbone(*ctx)
            begun = dp_begin(tf, cf, cams[0], not streams.enabled(device)) if _DP_BEGIN_SIDE else None
            return tf, cf, cams, begun

        ctx = (context["image"], context["intrinsics"], context["extrinsics"], context["near"], context["far"])
        if _DA_SIDE:  # A/B arrangement: Depth-Anything on the side stream, the backbone here
            da = streams.fork(device, depth_anything, context["image"])
            trans_features, cnn_features, (dp_cams, adapter_cams), begun = backbone_branch(*ctx)
            da_depth, out_feature = streams.join(da)
        else:
            bb = streams.fork(device, backbone_branch, *ctx)
            da_depth, out_feature = depth_anything(context["image"])
            trans_features, cnn_features, (dp_cams, adapter_cams), begun = streams.join(bb)
        if begun is None:
            begun = dp_begin(trans_features, cnn_features, dp_cams, True)
        dino_feature = out_feature.view(b, v, *out_feature.shape[1:])

        extra_info = {"images": rearrange(context["image"], "b v c h w -> (v b) c h w"), "scene_names": scene_names}
        gpp = self.cfg.gaussians_per_pixel
        with bench("encoder_4_depth_predictor"), self._dense():
            depths, densities, raw_gaussians = self.depth_predictor(
                trans_features, context["intrinsics"], context["extrinsics"], context["near"], context["far"],
                gaussians_per_pixel=gpp, deterministic=deterministic, extra_info=extra_info,
                cnn_features=cnn_features, da_depth=da_depth, dino_feature=dino_feature, benchmarker=benchmarker,
                cams=dp_cams, begun=begun)
        depths, densities, raw_gaussians = depths.float(), densities.float(), raw_gaussians.float()

        with bench("encoder_5_gaussian_adapter"):
            # fused: sub-pixel offsets, rays, means, covariances, SH mask + rotation, opacity
            srf = self.cfg.num_surfaces
            if srf != 1 or gpp != 1:
                raise NotImplementedError("TranSplat runs 1 surface and 1 Gaussian per pixel")
            x = self.cfg.opacity_mapping
            exponent = 2 ** (x.initial + min(global_step / x.warm_up, 1) * (x.final - x.initial))
            means, covariances, harmonics, opacities = self.gaussian_adapter(
                context["extrinsics"], context["intrinsics"], raw_gaussians, depths.reshape(b, v, h * w),
                densities.reshape(b, v, h * w), (h, w), opacity_exponent=exponent, gaussians_per_pixel=gpp,
                camera_consts=adapter_cams)
        if visualization_dump is not None:
            visualization_dump["depth"] = rearrange(depths, "b v (h w) srf s -> b v h w srf s", h=h, w=w)
        return Gaussians(means, covariances, harmonics, opacities)

    def get_data_shim(self):
        """(reference :355-371) crop to a multiple of shim_patch_size * downscale_factor."""
        patch = self.cfg.shim_patch_size * self.cfg.downscale_factor

        def data_shim(batch):
            from ...dataset_shims import apply_patch_shim

            return apply_patch_shim(batch, patch_size=patch)

        return data_shim
