"""Canonical, order-independent weight fill used to pin modules against golden vectors.

Every floating tensor in a module's state_dict is filled from a generator seeded by
(seed, crc32(name)), so the reference module (in the golden generator) and the rebuilt module
(in the tests) receive identical weights whenever their state_dict keys agree — which is
itself the drop-in check for checkpoint loading.
"""
from __future__ import annotations

import zlib

import torch


def _gen(seed: int, name: str) -> torch.Generator:
    return torch.Generator().manual_seed((seed * 1_000_003 + zlib.crc32(name.encode())) % (2**63))


def fill_tensor(name: str, t: torch.Tensor, seed: int) -> torch.Tensor:
    g = _gen(seed, name)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "running_var":
        return 0.5 + torch.rand(t.shape, generator=g)
    if leaf == "running_mean":
        return 0.1 * torch.randn(t.shape, generator=g)
    if t.dim() >= 2:
        fan_in = max(1, t[0].numel())
        return torch.randn(t.shape, generator=g) / fan_in**0.5
    if leaf in ("weight", "gamma"):
        return 1.0 + 0.1 * torch.randn(t.shape, generator=g)
    return 0.1 * torch.randn(t.shape, generator=g)


@torch.no_grad()
def canonical_init(module: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    sd = module.state_dict()
    new = {}
    for name, t in sd.items():
        if torch.is_floating_point(t):
            new[name] = fill_tensor(name, t, seed).to(t.dtype)
        else:
            new[name] = t
    module.load_state_dict(new, strict=True)
    return module


def seeded(shape, seed: int, scale: float = 1.0, kind: str = "randn") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    if kind == "rand":
        return torch.rand(shape, generator=g) * scale
    return torch.randn(shape, generator=g) * scale
