"""ctypes front end of oracle/raster_ref.c (TEST INFRASTRUCTURE ONLY).

`render(...)` renders every view with the scalar C restatement of the graphdeco forward
rasterizer (see the header of raster_ref.c for the reference citations). Two arithmetic modes:
  * "literal" (default): the upstream source's own expressions -- glm-order EWA covariance, double
    ndc2Pix, power = -0.5f*(a dx^2 + c dy^2) - b dx dy, libm expf -- independent of the HIP kernel;
  * "kernel": the op order of the round-2 kernel (Horner power, Cephes exp), kept for regression
    of the oracle itself (test_oracle_modes_agree).
`render_flagged(...)` is the literal mode plus the threshold flags: per pixel, whether any blend
decision (power > 0, alpha >= 1/255, T < 1e-4, an ambiguous tile rect / radius / cull) lies
within a rounding margin of its threshold, and per Gaussian, whether its radius / rect / cull is
ambiguous. Parity tests exclude exactly the flagged pixels (and radii) and report their number.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

FLAG_RECT, FLAG_POWER, FLAG_ALPHA, FLAG_T = 1, 2, 4, 8

HERE = Path(__file__).resolve().parent
# TSPLAT_ORACLE_LIB: an alternative build of the same restatement (the ASan / UBSan one, `make asan`)
LIB = Path(os.environ.get("TSPLAT_ORACLE_LIB") or HERE / "build" / "libtsplat_oracle.so")
_lib = None


def build() -> Path:
    if os.environ.get("TSPLAT_ORACLE_LIB"):
        return LIB
    if not LIB.exists() or LIB.stat().st_mtime < (HERE / "raster_ref.c").stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(str(LIB))
        f = lib.tsplat_ref_raster_view
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 12
        f = lib.tsplat_ref_raster_view_literal
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 14
        lib.tsplat_ref_set_threads.argtypes = [ctypes.c_int]
        lib.tsplat_ref_set_threads.restype = None
        lib.tsplat_ref_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the C rasterizer (images are bit-identical for any count); returns the
    count in effect."""
    lib = load()
    lib.tsplat_ref_set_threads(int(n))
    return int(lib.tsplat_ref_max_threads())


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _render(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree,
            mode, flags):
    lib = load()
    f32 = lambda t: np.ascontiguousarray(np.asarray(t, dtype=np.float32))
    means, covariances, harmonics, opacities = map(f32, (means, covariances, harmonics, opacities))
    vm, pm, cp, tf, bg, sc = (f32(getattr(cams, k)) for k in ("viewmat", "projmat", "campos", "tanfov", "bg", "scale"))
    s, g = opacities.shape
    m = harmonics.shape[-1]
    h, w = image_shape
    v = vm.shape[0]
    color = np.zeros((v, 3, h, w), np.float32)
    radii = np.zeros((v, g), np.int32)
    pflag = np.zeros((v, h, w), np.uint8)
    gflag = np.zeros((v, g), np.uint8)
    counts = []
    for i in range(v):
        sc_i = i // views_per_scene
        out_c = np.zeros((3, h, w), np.float32)
        out_r = np.zeros((g,), np.int32)
        args = [g, h, w, m, sh_degree,
                _p(means[sc_i]), _p(covariances[sc_i]), _p(harmonics[sc_i]), _p(opacities[sc_i]),
                _p(vm[i]), _p(pm[i]), _p(cp[i]), _p(tf[i]), _p(bg[i]), _p(sc[i]), _p(out_c), _p(out_r)]
        if mode == "kernel":
            n = lib.tsplat_ref_raster_view(*args)
        elif mode == "literal":
            pf = np.zeros((h, w), np.uint8) if flags else None
            gf = np.zeros((g,), np.uint8) if flags else None
            n = lib.tsplat_ref_raster_view_literal(*args, _p(pf), _p(gf))
            if flags:
                pflag[i], gflag[i] = pf, gf
        else:
            raise ValueError(f"unknown oracle mode {mode!r}")
        if n < 0:
            raise MemoryError("oracle rasterizer allocation failed")
        counts.append(n)
        color[i], radii[i] = out_c, out_r
    return color, radii, counts, pflag, gflag.astype(bool)


def render(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree,
           mode: str = "literal"):
    """numpy/torch-CPU inputs in the tsplat_raster_fwd layouts -> (color [V,3,H,W], radii [V,G],
    instance counts per view)."""
    return _render(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree,
                   mode, False)[:3]


def render_flagged(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree):
    """Literal mode + threshold flags -> (color, radii, counts, pixel_flags [V,H,W] uint8,
    gaussian_flags [V,G] bool). Pixel flag bits: 1 ambiguous tile rect / radius / cull, 2 power
    near 0, 4 alpha near 1/255, 8 T near 1e-4 (FLAG_* below); 0 = every decision is clear."""
    return _render(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree,
                   "literal", True)
