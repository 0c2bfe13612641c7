"""Batch shim on the test path (reference src/dataset/shims/patch_shim.py:4-38): centre-crop the
images to a multiple of the patch size and rescale fx, fy accordingly."""
from __future__ import annotations


def apply_patch_shim_to_views(views: dict, patch_size: int) -> dict:
    _, _, _, h, w = views["image"].shape
    assert h % 2 == 0 and w % 2 == 0
    h_new = (h // patch_size) * patch_size
    row = (h - h_new) // 2
    w_new = (w // patch_size) * patch_size
    col = (w - w_new) // 2
    intrinsics = views["intrinsics"].clone()
    intrinsics[:, :, 0, 0] *= w / w_new
    intrinsics[:, :, 1, 1] *= h / h_new
    return {**views, "image": views["image"][:, :, :, row:row + h_new, col:col + w_new], "intrinsics": intrinsics}


def apply_patch_shim(batch: dict, patch_size: int) -> dict:
    return {**batch, "context": apply_patch_shim_to_views(batch["context"], patch_size),
            "target": apply_patch_shim_to_views(batch["target"], patch_size)}
