"""Camera setup + call of the gfx950 Gaussian rasterizer (replaces reference `render_cuda`).

Reference: src/model/decoder/cuda_splatting.py:26-136. The reference repeats the Gaussians
over every target view, then loops the views in Python (two `.item()` host syncs per view) and
calls the third-party CUDA rasterizer once per view. Here the per-view camera constants are
computed once on the device (same torch expressions as the reference) and every view of every
scene is rasterized by one `tsplat_raster_fwd` call that reads the un-repeated Gaussian buffers.
"""
from __future__ import annotations

from dataclasses import dataclass
from math import isqrt

import torch
from torch import Tensor

from ... import kernels
from ... import _lib
from ...geometry.projection import get_fov


def get_projection_matrix(near: Tensor, far: Tensor, fov_x: Tensor, fov_y: Tensor) -> Tensor:
    """(reference cuda_splatting.py:26-53) x/y -> (-1, 1), z -> (0, 1)."""
    tan_fov_x = (0.5 * fov_x).tan()
    tan_fov_y = (0.5 * fov_y).tan()
    top = tan_fov_y * near
    bottom = -top
    right = tan_fov_x * near
    left = -right
    (b,) = near.shape
    result = torch.zeros((b, 4, 4), dtype=torch.float32, device=near.device)
    result[:, 0, 0] = 2 * near / (right - left)
    result[:, 1, 1] = 2 * near / (top - bottom)
    result[:, 0, 2] = (right + left) / (right - left)
    result[:, 1, 2] = (top + bottom) / (top - bottom)
    result[:, 3, 2] = 1
    result[:, 2, 2] = far / (far - near)
    result[:, 2, 3] = -(far * near) / (far - near)
    return result


@dataclass
class RasterCameras:
    """Per-view constants in the layouts of `tsplat_raster_fwd` (all fp32, contiguous)."""

    viewmat: Tensor  # [V, 16] column-major view matrix (= inverse(c2w)^T row-major)
    projmat: Tensor  # [V, 16] column-major full projection
    campos: Tensor  # [V, 3]
    tanfov: Tensor  # [V, 2]
    bg: Tensor  # [V, 3]
    scale: Tensor  # [V, 2] (s, s^2), s = 1/near when scale-invariant, else 1

    def to(self, device) -> "RasterCameras":
        return RasterCameras(*(getattr(self, f).to(device) for f in self.__dataclass_fields__))


def prepare_cameras(
    extrinsics: Tensor,
    intrinsics: Tensor,
    near: Tensor,
    far: Tensor,
    background_color: Tensor,
    scale_invariant: bool = True,
) -> RasterCameras:
    """Camera math of render_cuda (cuda_splatting.py:73-96) for V = (b v) flattened views. Device
    tensors: one launch (tsplat_raster_cameras); host tensors (the oracle / CPU-baseline callers)
    take the same math on torch ops."""
    if extrinsics.is_cuda:
        lib = _lib.load()
        v = extrinsics.shape[0]
        dev = extrinsics.device
        f = lambda t: t.float().contiguous()
        ext, intr, nr, fr, bg = f(extrinsics), f(intrinsics), f(near), f(far), f(background_color)
        out = [torch.empty((v, n), dtype=torch.float32, device=dev) for n in (16, 16, 3, 2, 3, 2)]
        rc = lib.tsplat_raster_cameras(_lib.ptr(ext), _lib.ptr(intr), _lib.ptr(nr), _lib.ptr(fr), _lib.ptr(bg),
                                       int(bg.dim() == 2), int(scale_invariant), v, *(_lib.ptr(t) for t in out),
                                       _lib.stream_ptr(dev))
        _lib.check(rc, "tsplat_raster_cameras")
        return RasterCameras(*out)
    extrinsics = extrinsics.float()
    if scale_invariant:
        scale = 1 / near
        extrinsics = extrinsics.clone()
        extrinsics[..., :3, 3] = extrinsics[..., :3, 3] * scale[:, None]
        near = near * scale
        far = far * scale
    else:
        scale = torch.ones_like(near)
    fov_x, fov_y = get_fov(intrinsics).unbind(dim=-1)
    tan_fov_x = (0.5 * fov_x).tan()
    tan_fov_y = (0.5 * fov_y).tan()
    projection_matrix = get_projection_matrix(near, far, fov_x, fov_y).transpose(1, 2)
    view_matrix = kernels.small_inverse(extrinsics).transpose(1, 2)
    full_projection = view_matrix @ projection_matrix
    v = extrinsics.shape[0]
    return RasterCameras(
        viewmat=view_matrix.contiguous().view(v, 16),
        projmat=full_projection.contiguous().view(v, 16),
        campos=extrinsics[:, :3, 3].contiguous(),
        tanfov=torch.stack((tan_fov_x, tan_fov_y), dim=-1).contiguous(),
        bg=background_color.float().contiguous(),
        scale=torch.stack((scale, scale * scale), dim=-1).float().contiguous(),
    )


class _RasterState:
    """Per-device workspace + sticky overflow status, grown on demand. A superseded workspace is
    retired, not freed: a captured hipGraph may still hold its address."""

    def __init__(self):
        self.workspace: dict = {}
        self.status: dict = {}
        self.last: dict = {}
        self.retired: list = []

    def get(self, device, nbytes: int):
        key = (device.type, device.index)
        ws = self.workspace.get(key)
        if ws is None or ws.numel() < nbytes:
            if ws is not None:
                self.retired.append(ws)
            ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
            self.workspace[key] = ws
        st = self.status.get(key)
        if st is None:
            st = torch.zeros(1, dtype=torch.int32, device=device)
            self.status[key] = st
        return ws, st


_STATE = _RasterState()


MAX_CAPACITY = 1 << 30  # 8 GiB of 8-byte instance keys


def default_capacity(num_gaussians: int, num_views: int, height: int, width: int) -> int:
    """The worst case, every Gaussian touching every 16x16 tile of every view, so a captured
    graph can never overflow (the reference sizes its buffers from a host readback of the exact
    count instead, which a graph cannot do). 8 bytes per instance: 0.8 GB for one 256x256 scene
    x 3 views, 6.4 GB at batch 8, a small slice of 288 GB. Larger problems are capped at
    MAX_CAPACITY and rely on the overflow status."""
    tiles = ((height + 15) // 16) * ((width + 15) // 16)
    return max(1, min(num_gaussians * num_views * tiles, MAX_CAPACITY))


def rasterize(
    means: Tensor,
    covariances: Tensor,
    harmonics: Tensor,
    opacities: Tensor,
    cameras: RasterCameras,
    image_shape: tuple[int, int],
    views_per_scene: int,
    sh_degree: int | None = None,
    capacity: int | None = None,
    check: bool = True,
    debug: bool = False,
) -> tuple[Tensor, Tensor]:
    """Render V = scenes * views_per_scene views.

    debug=True mirrors the upstream rasterizer's `debug` setting (cuda_splatting.py:120): every
    launch of the call is followed by a device synchronisation and an error check
    (tsplat_set_debug), so a faulting kernel is named; it cannot run inside hipGraph capture.

    means [S, G, 3], covariances [S, G, 3, 3], harmonics [S, G, 3, M], opacities [S, G]
    -> color [V, 3, H, W], radii [V, G] int32.
    `sh_degree` defaults to isqrt(M) - 1 (the degree render_cuda passes) capped at the
    evaluated degree of the upstream rasterizer (3); pass 4 to evaluate degree-4 terms.
    """
    lib = _lib.load()
    s, g, _ = means.shape
    m = harmonics.shape[-1]
    v = cameras.viewmat.shape[0]
    if v != s * views_per_scene:
        raise ValueError(f"{v} views for {s} scenes x {views_per_scene} views per scene")
    if covariances.shape != (s, g, 3, 3) or harmonics.shape[:3] != (s, g, 3) or opacities.shape != (s, g):
        raise ValueError("Gaussian tensor shapes disagree")
    if sh_degree is None:
        sh_degree = min(isqrt(m) - 1, 3)
    h, w = image_shape
    dev = means.device
    f32 = lambda t: t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()
    means, covariances, harmonics, opacities = map(f32, (means, covariances, harmonics, opacities))
    if capacity is None:
        capacity = default_capacity(g, v, h, w)
    nbytes = int(lib.tsplat_raster_workspace_bytes(g, v, h, w, capacity))
    ws, status = _STATE.get(dev, nbytes)
    color = torch.empty((v, 3, h, w), dtype=torch.float32, device=dev)
    radii = torch.empty((v, g), dtype=torch.int32, device=dev)
    desc = _lib.RasterDesc(g, v, views_per_scene, h, w, m, sh_degree, capacity)
    cams = [f32(cameras.viewmat), f32(cameras.projmat), f32(cameras.campos), f32(cameras.tanfov),
            f32(cameras.bg), f32(cameras.scale)]
    for t in cams:
        if t.device != dev:
            raise ValueError("camera tensors must be on the Gaussians' device")
    if debug and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("rasterize(debug=True) synchronises after every launch: not inside hipGraph capture")
    was = lib.tsplat_set_debug(1) if debug else None
    try:
        rc = lib.tsplat_raster_fwd(
            desc,
            *(_lib.ptr(t) for t in (means, covariances, harmonics, opacities)),
            *(_lib.ptr(t) for t in cams),
            _lib.ptr(color),
            _lib.ptr(radii),
            _lib.ptr(ws),
            _lib.ptr(status),
            _lib.stream_ptr(dev),
        )
    finally:
        if was is not None:
            lib.tsplat_set_debug(was)
    _lib.check(rc, "tsplat_raster_fwd")
    _STATE.last[(dev.type, dev.index)] = (ws, int(lib.tsplat_raster_num_rendered_offset(g, v, h, w)))
    if check:
        check_status(dev)
    return color, radii


def num_rendered(device) -> int:
    """(Gaussian, tile) instances generated by the last rasterize() on `device` (the reference
    forward's num_rendered; syncs)."""
    ws, off = _STATE.last[(device.type, device.index)]
    return int(ws[off:off + 4].view(torch.int32).item())


def status_tensor(device):
    """The device's sticky overflow flag (int32 [1]; None before the first rasterize) -- read
    without a sync by copying it on the stream."""
    return _STATE.status.get((device.type, device.index))


def check_status(device) -> None:
    """Raise if any rasterizer call on `device` overflowed its instance capacity (syncs)."""
    st = _STATE.status.get((device.type, device.index))
    if st is not None and int(st.item()) != 0:
        st.zero_()
        raise RuntimeError("tsplat_raster_fwd: instance capacity exceeded; pass a larger capacity")
