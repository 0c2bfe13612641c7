"""Encoder ABC (reference src/model/encoder/encoder.py:12-29)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Generic, TypeVar

from torch import nn

from ..types import Gaussians

T = TypeVar("T")


class Encoder(nn.Module, ABC, Generic[T]):
    cfg: T

    def __init__(self, cfg: T) -> None:
        super().__init__()
        self.cfg = cfg

    @abstractmethod
    def forward(self, context: dict, deterministic: bool) -> Gaussians:
        pass

    def get_data_shim(self):
        return lambda x: x
