"""Batch shim on the test path (reference src/dataset/shims/patch_shim.py:4-38): centre-crop the
images to a multiple of the patch size and rescale fx, fy accordingly."""
from __future__ import annotations

import torch

_SCALES: dict = {}


def apply_patch_shim_to_views(views: dict, patch_size: int) -> dict:
    _, _, _, h, w = views["image"].shape
    assert h % 2 == 0 and w % 2 == 0
    h_new = (h // patch_size) * patch_size
    row = (h - h_new) // 2
    w_new = (w // patch_size) * patch_size
    col = (w - w_new) // 2
    k = views["intrinsics"]
    # fx *= w / w_new, fy *= h / h_new as ONE multiply by a cached [3, 3] scale (1 elsewhere: exact,
    # and the same fp32 product as the in-place scalar multiplies) instead of clone + two launches
    key = (k.device, k.dtype, k.shape[-1], w / w_new, h / h_new)
    scale = _SCALES.get(key)
    if scale is None:
        scale = torch.ones(k.shape[-2:], dtype=k.dtype, device=k.device)
        scale[0, 0] = w / w_new
        scale[1, 1] = h / h_new
        _SCALES[key] = scale
    return {**views, "image": views["image"][:, :, :, row:row + h_new, col:col + w_new], "intrinsics": k * scale}


def apply_patch_shim(batch: dict, patch_size: int) -> dict:
    return {**batch, "context": apply_patch_shim_to_views(batch["context"], patch_size),
            "target": apply_patch_shim_to_views(batch["target"], patch_size)}
