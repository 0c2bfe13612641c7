"""`splatting_hip` decoder: drop-in for DecoderSplattingCUDA
(reference src/model/decoder/decoder_splatting_cuda.py:26-97).

Differences by design: the Gaussians are NOT repeated per target view (the reference
materialises V copies, 46 MB each at G = 131072); all (b v) views go to one rasterizer call.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Literal, Optional

import torch
from einops import rearrange, repeat
from torch import Tensor

from ..types import Gaussians
from .decoder import Decoder, DecoderOutput, DepthRenderingMode
from .hip_splatting import check_status, prepare_cameras, rasterize


@dataclass
class DecoderSplattingHIPCfg:
    name: Literal["splatting_hip", "splatting_cuda"] = "splatting_hip"
    sh_eval_degree: Optional[int] = None  # None: min(isqrt(d_sh) - 1, 3), the upstream behaviour
    check_overflow: bool = True  # sync after each call to surface capacity overflow
    debug: bool = False  # upstream GaussianRasterizationSettings.debug: sync + check after every launch


def depth_fake_color(extrinsics: Tensor, means: Tensor, near: Tensor, far: Tensor,
                     mode: DepthRenderingMode = "depth") -> Tensor:
    """Per-view fake colour of the depth render (reference cuda_splatting.py:388-401):
    extrinsics [V, 4, 4] c2w, means [V, G, 3], near / far [V] -> [V, G]. The "log" mode keeps the
    reference's minimum(near).maximum(far) order."""
    cam = torch.einsum("bij,bgj->bgi", extrinsics.inverse(), torch.cat([means, torch.ones_like(means[..., :1])], -1))
    fake = cam[..., 2]
    if mode == "disparity":
        fake = 1 / fake
    elif mode == "relative_disparity":
        eps = 1e-10  # depth_to_relative_disparity (reference matching/conversions.py:18-28)
        disp_near, disp_far = 1 / (near[:, None] + eps), 1 / (far[:, None] + eps)
        fake = 1 - (1 / (fake + eps) - disp_far) / (disp_near - disp_far + eps)
    elif mode == "log":
        fake = fake.minimum(near[:, None]).maximum(far[:, None]).log()
    return fake


class DecoderSplattingHIP(Decoder[DecoderSplattingHIPCfg]):
    background_color: Tensor

    def __init__(self, cfg: DecoderSplattingHIPCfg, dataset_cfg) -> None:
        super().__init__(cfg, dataset_cfg)
        self.register_buffer(
            "background_color",
            torch.tensor(dataset_cfg.background_color, dtype=torch.float32),
            persistent=False,
        )

    def forward(
        self,
        gaussians: Gaussians,
        extrinsics: Tensor,
        intrinsics: Tensor,
        near: Tensor,
        far: Tensor,
        image_shape: tuple[int, int],
        depth_mode: DepthRenderingMode | None = None,
    ) -> DecoderOutput:
        b, v, _, _ = extrinsics.shape
        cams = prepare_cameras(
            rearrange(extrinsics, "b v i j -> (b v) i j"),
            rearrange(intrinsics, "b v i j -> (b v) i j"),
            rearrange(near, "b v -> (b v)"),
            rearrange(far, "b v -> (b v)"),
            repeat(self.background_color, "c -> (b v) c", b=b, v=v),
        )
        color, _ = rasterize(
            gaussians.means,
            gaussians.covariances,
            gaussians.harmonics,
            gaussians.opacities,
            cams,
            image_shape,
            views_per_scene=v,
            sh_degree=self.cfg.sh_eval_degree,
            check=self.cfg.check_overflow,
            debug=self.cfg.debug,
        )
        color = rearrange(color, "(b v) c h w -> b v c h w", b=b, v=v)
        depth = None
        if depth_mode is not None:
            depth = self.render_depth(gaussians, extrinsics, intrinsics, near, far, image_shape, depth_mode)
        return DecoderOutput(color, depth)

    def render_depth(
        self,
        gaussians: Gaussians,
        extrinsics: Tensor,
        intrinsics: Tensor,
        near: Tensor,
        far: Tensor,
        image_shape: tuple[int, int],
        mode: DepthRenderingMode = "depth",
    ) -> Tensor:
        """Depth as fake colour (reference cuda_splatting.py:375-417); one call per view set."""
        b, v, _, _ = extrinsics.shape
        ext = rearrange(extrinsics, "b v i j -> (b v) i j")
        means = repeat(gaussians.means, "b g xyz -> (b v) g xyz", v=v)
        nr = rearrange(near, "b v -> (b v)")
        fr = rearrange(far, "b v -> (b v)")
        fake = depth_fake_color(ext, means, nr, fr, mode)
        cams = prepare_cameras(ext, rearrange(intrinsics, "b v i j -> (b v) i j"), nr, fr,
                               torch.zeros((b * v, 3), device=ext.device))
        color, _ = rasterize(
            means,
            repeat(gaussians.covariances, "b g i j -> (b v) g i j", v=v),
            repeat(fake, "bv g -> bv g c ()", c=3).contiguous(),
            repeat(gaussians.opacities, "b g -> (b v) g", v=v),
            cams,
            image_shape,
            views_per_scene=1,
            sh_degree=0,
            check=self.cfg.check_overflow,
            debug=self.cfg.debug,
        )
        return rearrange(color.mean(dim=1), "(b v) h w -> b v h w", b=b, v=v)

    @staticmethod
    def check_overflow(device) -> None:
        check_status(device)
