"""Decoder ABC and output type (reference src/model/decoder/decoder.py:20-48)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Generic, Literal, Optional, TypeVar

from torch import Tensor, nn

from ..types import Gaussians

DepthRenderingMode = Literal["depth", "log", "disparity", "relative_disparity"]


@dataclass
class DecoderOutput:
    color: Tensor  # [batch, view, 3, height, width]
    depth: Optional[Tensor]  # [batch, view, height, width] or None


@dataclass
class DatasetCfgLite:
    """The fields of the reference DatasetCfg a decoder reads (background colour)."""

    background_color: tuple = (0.0, 0.0, 0.0)


T = TypeVar("T")


class Decoder(nn.Module, ABC, Generic[T]):
    cfg: T

    def __init__(self, cfg: T, dataset_cfg) -> None:
        super().__init__()
        self.cfg = cfg
        self.dataset_cfg = dataset_cfg

    @abstractmethod
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
        pass
