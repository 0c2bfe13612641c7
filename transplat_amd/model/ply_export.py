"""Gaussian scene -> .ply (reference src/model/ply_export.py:12-92; same attribute list, scene
normalisation, viewer rotation, quaternion handling and DC-only colours).

`plyfile` is not a dependency here: the binary little-endian PLY (one `vertex` element, float32
properties in the reference's order) is written directly, and `read_ply` parses it back.
Visualisation / export only; not on the measured hot path.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch
from einops import einsum
from scipy.spatial.transform import Rotation as R
from torch import Tensor


def construct_list_of_attributes(num_rest: int) -> list[str]:
    """(reference :12-23)"""
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)]
    names += [f"f_rest_{i}" for i in range(num_rest)]
    names += ["opacity"] + [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]
    return names


def ply_vertices(extrinsics: Tensor, means: Tensor, scales: Tensor, rotations: Tensor, harmonics: Tensor,
                 opacities: Tensor) -> np.ndarray:
    """The structured vertex array the reference hands PlyElement.describe (reference :26-88):
    means centred on their median and scaled by the max over axes of the 95 % quantile of |mean|,
    rotated into a +Z-up, 45-degree-adjusted frame composed with the w2c rotation; rotations
    (xyzw) rotated likewise and written wxyz; DC band of the harmonics; log scales; raw opacity."""
    means = means - means.median(dim=0).values
    scale_factor = means.abs().quantile(0.95, dim=0).max()
    means = means / scale_factor
    scales = scales / scale_factor
    rotation = torch.tensor([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=torch.float32, device=means.device)
    adjustment = torch.tensor(R.from_rotvec([0, 0, -45], True).as_matrix(), dtype=torch.float32, device=means.device)
    rotation = adjustment @ rotation
    rotation = rotation @ extrinsics[:3, :3].inverse()
    means = einsum(rotation, means, "i j, ... j -> ... i")
    rot = R.from_quat(rotations.detach().cpu().numpy()).as_matrix()
    rot = rotation.detach().cpu().numpy() @ rot
    xyzw = R.from_matrix(rot).as_quat()
    wxyz = np.stack((xyzw[:, 3], xyzw[:, 0], xyzw[:, 1], xyzw[:, 2]), axis=-1)
    dtype = [(name, "f4") for name in construct_list_of_attributes(0)]
    cols = np.concatenate((
        means.detach().cpu().numpy(),
        np.zeros((means.shape[0], 3), np.float32),
        harmonics[..., 0].detach().cpu().contiguous().numpy(),
        opacities[..., None].detach().cpu().numpy(),
        scales.log().detach().cpu().numpy(),
        wxyz,
    ), axis=1)
    out = np.empty(means.shape[0], dtype=dtype)
    for i, (name, _) in enumerate(dtype):
        out[name] = cols[:, i]
    return out


def write_ply(vertices: np.ndarray, path: Path) -> None:
    """Binary little-endian PLY with one `vertex` element of float32 properties."""
    path = Path(path)
    path.parent.mkdir(exist_ok=True, parents=True)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {len(vertices)}"]
    header += [f"property float {name}" for name in vertices.dtype.names] + ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(vertices.astype(vertices.dtype.newbyteorder("<")).tobytes())


def read_ply(path: Path) -> np.ndarray:
    """Parse a file written by write_ply (float32 vertex properties only)."""
    data = Path(path).read_bytes()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    lines = data[:end].decode("ascii").splitlines()
    if lines[0] != "ply" or lines[1] != "format binary_little_endian 1.0":
        raise ValueError("not a binary little-endian PLY written by write_ply")
    n = int(next(l for l in lines if l.startswith("element vertex")).split()[-1])
    names = [l.split()[-1] for l in lines if l.startswith("property float")]
    return np.frombuffer(data[end:], dtype=[(name, "<f4") for name in names], count=n)


def export_ply(extrinsics: Tensor, means: Tensor, scales: Tensor, rotations: Tensor, harmonics: Tensor,
               opacities: Tensor, path: Path) -> None:
    """(reference :26-92) same signature; the scene for one context camera `extrinsics` [4, 4]."""
    write_ply(ply_vertices(extrinsics, means, scales, rotations, harmonics, opacities), path)
