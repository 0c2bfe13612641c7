"""Camera helpers on the hot path (reference src/geometry/projection.py).

Only the functions the encoder -> adapter -> decoder path calls are restated: `get_fov`
(:233-247), `sample_image_grid` (:117-137), `get_world_rays` (:91-114) and their helpers.
"""
from __future__ import annotations

import torch
from einops import einsum
from torch import Tensor
from .. import kernels


def homogenize_points(points: Tensor) -> Tensor:
    return torch.cat([points, torch.ones_like(points[..., :1])], dim=-1)


def homogenize_vectors(vectors: Tensor) -> Tensor:
    return torch.cat([vectors, torch.zeros_like(vectors[..., :1])], dim=-1)


def transform_rigid(homogeneous_coordinates: Tensor, transformation: Tensor) -> Tensor:
    return einsum(transformation, homogeneous_coordinates, "... i j, ... j -> ... i")


def transform_cam2world(homogeneous_coordinates: Tensor, extrinsics: Tensor) -> Tensor:
    return transform_rigid(homogeneous_coordinates, extrinsics)


def unproject(coordinates: Tensor, z: Tensor, intrinsics: Tensor) -> Tensor:
    coordinates = homogenize_points(coordinates)
    ray_directions = einsum(kernels.small_inverse(intrinsics), coordinates, "... i j, ... j -> ... i")
    return ray_directions * z[..., None]


def get_world_rays(coordinates: Tensor, extrinsics: Tensor, intrinsics: Tensor):
    """(reference projection.py:91-114) unit world-space ray directions and camera origins."""
    directions = unproject(coordinates, torch.ones_like(coordinates[..., 0]), intrinsics)
    directions = directions / directions.norm(dim=-1, keepdim=True)
    directions = homogenize_vectors(directions)
    directions = transform_cam2world(directions, extrinsics)[..., :-1]
    origins = extrinsics[..., :-1, -1].broadcast_to(directions.shape)
    return origins, directions


def sample_image_grid(shape: tuple[int, ...], device: torch.device = torch.device("cpu")):
    """(reference projection.py:117-137) pixel-centre coordinates in (0, 1), xy order."""
    indices = [torch.arange(length, device=device) for length in shape]
    stacked_indices = torch.stack(torch.meshgrid(*indices, indexing="ij"), dim=-1)
    coordinates = [(idx + 0.5) / length for idx, length in zip(indices, shape)]
    coordinates = reversed(coordinates)
    coordinates = torch.stack(torch.meshgrid(*coordinates, indexing="xy"), dim=-1)
    return coordinates, stacked_indices


_EDGE_MIDPOINTS: dict = {}


def _edge_midpoints(device) -> Tensor:
    """left, right, top, bottom image-edge midpoints, cached per device so no host->device copy
    happens after the first call (graph-capture safe)."""
    key = (device.type, device.index)
    if key not in _EDGE_MIDPOINTS:
        _EDGE_MIDPOINTS[key] = torch.tensor([[0, 0.5, 1], [1, 0.5, 1], [0.5, 0, 1], [0.5, 1, 1]],
                                            dtype=torch.float32).to(device)
    return _EDGE_MIDPOINTS[key]


def get_fov(intrinsics: Tensor) -> Tensor:
    """(reference projection.py:233-247) fov from K^-1 applied to the edge midpoints."""
    intrinsics_inv = kernels.small_inverse(intrinsics)
    mids = _edge_midpoints(intrinsics.device)

    def process_vector(i):
        vector = einsum(intrinsics_inv, mids[i], "b i j, j -> b i")
        return vector / vector.norm(dim=-1, keepdim=True)

    left = process_vector(0)
    right = process_vector(1)
    top = process_vector(2)
    bottom = process_vector(3)
    fov_x = (left * right).sum(dim=-1).acos()
    fov_y = (top * bottom).sum(dim=-1).acos()
    return torch.stack((fov_x, fov_y), dim=-1)
