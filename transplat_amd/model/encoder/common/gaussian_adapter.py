"""Raw per-pixel head output -> world-space Gaussians (reference
src/model/encoder/common/gaussian_adapter.py:30-117), as one fused gfx950 kernel
(tsplat_gaussian_adapter_fwd); the torch expressions of the reference live in the oracle."""
from __future__ import annotations

from dataclasses import dataclass

import torch
from einops import einsum, rearrange
from torch import Tensor, nn

from .... import kernels


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

    def forward(self, extrinsics, intrinsics, raw_gaussians, depths, densities, image_shape,
                opacity_exponent: float = 1.0, gaussians_per_pixel: int = 1, camera_consts=None):
        """Fused stage 5 + adapter on the GPU (kernels.gaussian_adapter):
        raw [b, v, HW, 2 + d_in] head output, depths / densities [b, v, HW], cameras [b, v, ...]
        -> (means, covariances, harmonics, opacities) flattened to [b, v*HW, ...]."""
        extra = {"camera_consts": camera_consts} if camera_consts is not None else {}
        return kernels.gaussian_adapter(raw_gaussians, depths, densities, extrinsics, intrinsics, image_shape,
                                        self.cfg.gaussian_scale_min, self.cfg.gaussian_scale_max,
                                        opacity_exponent, gaussians_per_pixel, **extra)

    def get_scale_multiplier(self, intrinsics, pixel_size, multiplier: float = 0.1):
        xy_multipliers = multiplier * einsum(kernels.small_inverse(intrinsics[..., :2, :2].contiguous()), pixel_size, "... i j, j -> ... i")
        return xy_multipliers.sum(dim=-1)

    @property
    def d_sh(self) -> int:
        return (self.cfg.sh_degree + 1) ** 2

    @property
    def d_in(self) -> int:
        return 7 + 3 * self.d_sh
