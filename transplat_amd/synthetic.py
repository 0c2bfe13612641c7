"""Synthetic scenes for benchmarks and parity tests.

No dataset or checkpoint is reachable offline, so every workload is generated here:
  * context images U[0, 1) [b, V, 3, H, W];
  * normalised intrinsics fx = fy = 1, cx = cy = 0.5 for context and target views;
  * context c2w: view 0 = I, view 1 = translation (1, 0, 0) + 5 deg yaw (view k: k x that step);
    the 3 targets interpolate between views 0 and 1 at t in {0.25, 0.5, 0.75};
  * near = 1, far = 100 (re10k / ACID, reference config/experiment/re10k.yaml:40-41);
  * seed = 20260320 + scene_id through a CPU torch.Generator, then moved to the device.
`make_gaussians` builds rasterizer-only inputs: per-pixel depth U[2, 20] on the context views,
means = ray * depth, covariance R S S^T R^T from N(0, 1) raw scale/rotation features through
the adapter's maps, SH ~ N(0, 1) * sh_mask, opacity U(0, 1).
"""
from __future__ import annotations

import math

import torch

BASE_SEED = 20260320


def _yaw(deg: float) -> torch.Tensor:
    a = math.radians(deg)
    r = torch.eye(4)
    r[0, 0], r[0, 2], r[2, 0], r[2, 2] = math.cos(a), math.sin(a), -math.sin(a), math.cos(a)
    return r


def context_extrinsics(num_views: int = 2, step: float = 1.0, yaw_deg: float = 5.0) -> torch.Tensor:
    ext = []
    for k in range(num_views):
        e = _yaw(yaw_deg * k)
        e[0, 3] = step * k
        ext.append(e)
    return torch.stack(ext)


def target_extrinsics(ctx: torch.Tensor, ts=(0.25, 0.5, 0.75)) -> torch.Tensor:
    out = []
    for t in ts:
        e = _yaw(5.0 * t)
        e[:3, 3] = (1 - t) * ctx[0, :3, 3] + t * ctx[1, :3, 3]
        out.append(e)
    return torch.stack(out)


def intrinsics(n: int) -> torch.Tensor:
    k = torch.tensor([[1.0, 0.0, 0.5], [0.0, 1.0, 0.5], [0.0, 0.0, 1.0]])
    return k.expand(n, 3, 3).clone()


def make_batch(
    batch: int,
    num_context: int = 2,
    num_target: int = 3,
    image_shape=(256, 256),
    scene_offset: int = 0,
    device="cpu",
    near: float = 1.0,
    far: float = 100.0,
    target_ts=None,
) -> dict:
    """A `BatchedExample`-like dict with 'context' and 'target' views for `batch` scenes.
    `target_ts` places the targets along the context baseline (default evenly spaced)."""
    h, w = image_shape
    ctx_imgs, tgt_imgs = [], []
    for i in range(batch):
        gen = torch.Generator().manual_seed(BASE_SEED + scene_offset + i)
        ctx_imgs.append(torch.rand((num_context, 3, h, w), generator=gen))
        tgt_imgs.append(torch.rand((num_target, 3, h, w), generator=gen))
    ctx_ext = context_extrinsics(num_context)
    ts = tuple(target_ts) if target_ts is not None else tuple((k + 1) / (num_target + 1) for k in range(num_target))
    tgt_ext = target_extrinsics(ctx_ext, ts)

    def views(imgs, ext, n):
        return {
            "image": torch.stack(imgs).to(device),
            "extrinsics": ext.expand(batch, n, 4, 4).clone().to(device),
            "intrinsics": intrinsics(n).expand(batch, n, 3, 3).clone().to(device),
            "near": torch.full((batch, n), near, device=device),
            "far": torch.full((batch, n), far, device=device),
        }

    return {
        "context": views(ctx_imgs, ctx_ext, num_context),
        "target": views(tgt_imgs, tgt_ext, num_target),
        "scene": [f"synthetic_{scene_offset + i:06d}" for i in range(batch)],
    }


def sh_mask(sh_degree: int) -> torch.Tensor:
    """(reference gaussian_adapter.py:40-46) 1 for l = 0, 0.1 * 0.25^l above."""
    d_sh = (sh_degree + 1) ** 2
    mask = torch.ones(d_sh)
    for degree in range(1, sh_degree + 1):
        mask[degree**2 : (degree + 1) ** 2] = 0.1 * 0.25**degree
    return mask


def quaternion_to_matrix(q: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """xyzw (scipy order) quaternion -> rotation (reference gaussians.py:7-29)."""
    i, j, k, r = torch.unbind(q, dim=-1)
    two_s = 2 / ((q * q).sum(dim=-1) + eps)
    o = torch.stack(
        (
            1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
            two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
            two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
        ),
        -1,
    )
    return o.reshape(*q.shape[:-1], 3, 3)


def make_gaussians(
    scenes: int,
    num_context: int = 2,
    image_shape=(256, 256),
    sh_degree: int = 4,
    depth_range=(2.0, 20.0),
    scene_offset: int = 0,
    scale_range=(0.5, 15.0),
    device="cpu",
):
    """Rasterizer inputs (means, covariances, harmonics, opacities) of [scenes, V*H*W, ...]."""
    h, w = image_shape
    d_sh = (sh_degree + 1) ** 2
    out = {"means": [], "covariances": [], "harmonics": [], "opacities": []}
    ext = context_extrinsics(num_context)
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    xy = torch.stack([(xs + 0.5) / w, (ys + 0.5) / h], -1).reshape(-1, 2)
    k_inv = torch.linalg.inv(intrinsics(1)[0])
    dirs_cam = torch.cat([xy, torch.ones_like(xy[:, :1])], -1) @ k_inv.T
    dirs_cam = dirs_cam / dirs_cam.norm(dim=-1, keepdim=True)
    mult = 0.1 * (k_inv[:2, :2] @ torch.tensor([1.0 / w, 1.0 / h])).sum()
    for s in range(scenes):
        gen = torch.Generator().manual_seed(BASE_SEED + 7919 + scene_offset + s)
        means, covs = [], []
        for v in range(num_context):
            depth = depth_range[0] + (depth_range[1] - depth_range[0]) * torch.rand(h * w, generator=gen)
            rot = ext[v, :3, :3]
            dirs = dirs_cam @ rot.T
            means.append(ext[v, :3, 3] + dirs * depth[:, None])
            raw_s = torch.randn((h * w, 3), generator=gen)
            raw_q = torch.randn((h * w, 4), generator=gen)
            scale = scale_range[0] + (scale_range[1] - scale_range[0]) * raw_s.sigmoid()
            scale = scale * depth[:, None] * mult
            q = raw_q / (raw_q.norm(dim=-1, keepdim=True) + 1e-8)
            r = quaternion_to_matrix(q)
            sdiag = torch.diag_embed(scale)
            cov = r @ sdiag @ sdiag.transpose(-1, -2) @ r.transpose(-1, -2)
            covs.append(rot @ cov @ rot.T)
        n = num_context * h * w
        out["means"].append(torch.cat(means))
        out["covariances"].append(torch.cat(covs))
        out["harmonics"].append(torch.randn((n, 3, d_sh), generator=gen) * sh_mask(sh_degree))
        out["opacities"].append(torch.rand(n, generator=gen))
    return {k: torch.stack(v).to(device).contiguous() for k, v in out.items()}


@torch.no_grad()
def init_synthetic_weights(module: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    """Deterministic stand-in weights (no checkpoint offline): fan-in scaled normal for matrices
    and kernels, ~1 for norm scales, small biases, BN running stats near identity. Keeps every
    activation O(1) through the 110 M-parameter encoder so the workload (and its NaN-free
    numerics, e.g. the Depth-Anything min-max normalisation) matches a trained model's."""
    gen = torch.Generator().manual_seed(seed)
    for name, t in module.state_dict().items():
        if not torch.is_floating_point(t):
            continue
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "running_var":
            new = 0.5 + torch.rand(t.shape, generator=gen)
        elif leaf == "running_mean":
            new = 0.1 * torch.randn(t.shape, generator=gen)
        elif t.dim() >= 2:
            new = torch.randn(t.shape, generator=gen) / max(1, t[0].numel()) ** 0.5
        elif leaf in ("weight", "gamma"):
            new = 1.0 + 0.1 * torch.randn(t.shape, generator=gen)
        else:
            new = 0.1 * torch.randn(t.shape, generator=gen)
        t.copy_(new.to(t.dtype))
    return module
