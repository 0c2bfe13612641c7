"""PSNR as the reference computes it (reference src/evaluation/metrics.py:11-19)."""
from __future__ import annotations

import torch


@torch.no_grad()
def compute_psnr(ground_truth: torch.Tensor, predicted: torch.Tensor) -> torch.Tensor:
    """[batch, 3, H, W] pairs -> per-image PSNR: clip to [0, 1], per-image MSE, -10 log10."""
    ground_truth = ground_truth.clip(min=0, max=1)
    predicted = predicted.clip(min=0, max=1)
    mse = ((ground_truth - predicted) ** 2).flatten(1).mean(dim=-1)
    return -10 * mse.log10()
