"""Raw per-pixel head output -> world-space Gaussians (reference
src/model/encoder/common/gaussian_adapter.py:30-117)."""
from __future__ import annotations

from dataclasses import dataclass

import torch
from einops import einsum, rearrange
from torch import Tensor, nn

from ....geometry.projection import get_world_rays
from ....misc.sh_rotation import rotate_sh, sh_rotation_matrix
from .gaussians import build_covariance


@dataclass
class Gaussians:
    means: Tensor
    covariances: Tensor
    scales: Tensor
    rotations: Tensor
    harmonics: Tensor
    opacities: Tensor


@dataclass
class GaussianAdapterCfg:
    gaussian_scale_min: float = 0.5
    gaussian_scale_max: float = 15.0
    sh_degree: int = 4


class GaussianAdapter(nn.Module):
    def __init__(self, cfg: GaussianAdapterCfg):
        super().__init__()
        self.cfg = cfg
        self.register_buffer("sh_mask", torch.ones((self.d_sh,), dtype=torch.float32), persistent=False)
        for degree in range(1, self.cfg.sh_degree + 1):
            self.sh_mask[degree**2:(degree + 1) ** 2] = 0.1 * 0.25**degree

    def forward(self, extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians, image_shape,
                eps: float = 1e-8) -> Gaussians:
        device = extrinsics.device
        scales, rotations, sh = raw_gaussians.split((3, 4, 3 * self.d_sh), dim=-1)
        scales = self.cfg.gaussian_scale_min + (self.cfg.gaussian_scale_max - self.cfg.gaussian_scale_min) * scales.sigmoid()
        h, w = image_shape
        pixel_size = 1 / torch.tensor((w, h), dtype=torch.float32, device=device)
        multiplier = self.get_scale_multiplier(intrinsics, pixel_size)
        scales = scales * depths[..., None] * multiplier[..., None]
        rotations = rotations / (rotations.norm(dim=-1, keepdim=True) + eps)
        sh = rearrange(sh, "... (xyz d_sh) -> ... xyz d_sh", xyz=3)
        sh = sh.broadcast_to((*opacities.shape, 3, self.d_sh)) * self.sh_mask
        covariances = build_covariance(scales, rotations)
        c2w_rotations = extrinsics[..., :3, :3]
        covariances = c2w_rotations @ covariances @ c2w_rotations.transpose(-1, -2)
        origins, directions = get_world_rays(coordinates, extrinsics, intrinsics)
        means = origins + directions * depths[..., None]
        return Gaussians(
            means=means,
            covariances=covariances,
            harmonics=self.rotate_harmonics(sh, c2w_rotations),
            opacities=opacities,
            scales=scales,
            rotations=rotations.broadcast_to((*scales.shape[:-1], 4)),
        )

    @staticmethod
    def rotate_harmonics(sh, c2w_rotations):
        """rotate_sh(sh, R[..., None, :, :]) with one D matrix per camera applied as a batched
        GEMM over the pixels (no per-pixel broadcast of D)."""
        b, v = sh.shape[:2]
        if c2w_rotations.shape[:2] == (b, v) and all(s == 1 for s in c2w_rotations.shape[2:-2]):
            d = sh_rotation_matrix(c2w_rotations.reshape(b, v, 3, 3), sh.shape[-1]).to(sh.dtype)
            flat = sh.reshape(b, v, -1, sh.shape[-1])
            return torch.einsum("bvij,bvnj->bvni", d, flat).reshape(sh.shape)
        return rotate_sh(sh, c2w_rotations[..., None, :, :])

    def get_scale_multiplier(self, intrinsics, pixel_size, multiplier: float = 0.1):
        xy_multipliers = multiplier * einsum(intrinsics[..., :2, :2].inverse(), pixel_size, "... i j, j -> ... i")
        return xy_multipliers.sum(dim=-1)

    @property
    def d_sh(self) -> int:
        return (self.cfg.sh_degree + 1) ** 2

    @property
    def d_in(self) -> int:
        return 7 + 3 * self.d_sh
