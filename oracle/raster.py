"""ctypes front end of oracle/raster_ref.c (TEST INFRASTRUCTURE ONLY).

`render(...)` renders every view with the scalar C restatement of the graphdeco forward
rasterizer (see the header of raster_ref.c for the reference citations).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libtsplat_oracle.so"
_lib = None


def build() -> Path:
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


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def render(means, covariances, harmonics, opacities, cams, image_shape, views_per_scene, sh_degree):
    """numpy/torch-CPU inputs in the tsplat_raster_fwd layouts -> (color [V,3,H,W], radii [V,G])."""
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
    counts = []
    for i in range(v):
        sc_i = i // views_per_scene
        out_c = np.zeros((3, h, w), np.float32)
        out_r = np.zeros((g,), np.int32)
        n = lib.tsplat_ref_raster_view(
            g, h, w, m, sh_degree,
            _p(means[sc_i]), _p(covariances[sc_i]), _p(harmonics[sc_i]), _p(opacities[sc_i]),
            _p(vm[i]), _p(pm[i]), _p(cp[i]), _p(tf[i]), _p(bg[i]), _p(sc[i]), _p(out_c), _p(out_r),
        )
        if n < 0:
            raise MemoryError("oracle rasterizer allocation failed")
        counts.append(n)
        color[i], radii[i] = out_c, out_r
    return color, radii, counts
