"""e3nn-free rotation of real spherical-harmonic coefficients (reference src/misc/sh_rotation.py:10-30).

The reference computes `alpha, beta, gamma = e3nn.o3.matrix_to_angles(R)` and applies
`e3nn.o3.wigner_D(l, alpha, beta, gamma)` to each degree block of the coefficients. e3nn is not
available (and its version is unpinned), so its published construction is restated:
  * su(2) generators of spin l, conjugated into e3nn's real basis (change_basis_real_to_complex,
    with the (-i)^l phase, which cancels) -> real so(3) generators X_x, X_y, X_z;
  * wigner_D = exp(alpha X_y) exp(beta X_x) exp(gamma X_y)  (Y-X-Y Euler angles);
  * matrix_to_angles: beta/alpha from R e_y (xyz_to_angles), gamma from the residual rotation.
The restated construction gives D^1 = R itself in e3nn's real basis, and that is what
tests/test_sh_rotation.py asserts, together with the representation properties (orthogonality,
D(R1 R2) = D(R1) D(R2)) for l <= 4. The reference's own, unasserted script
(src/misc/fast_sh_rotation.py:56-60,217-228) claims D^1 = R with rows and columns permuted to
(y, z, x) instead; the two disagree, and which convention the trained checkpoint saw cannot be settled
without e3nn (absent, version unpinned): A4 is "parity unpinned" against e3nn itself.
The D matrices are built per camera in float64 (a handful of 9x9 exponentials) and applied to the
per-pixel coefficients as one batched contraction.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch


@lru_cache(maxsize=None)
def _so3_generators(l: int) -> torch.Tensor:
    """[3, 2l+1, 2l+1] float64 real generators (e3nn so3_generators)."""
    j = l
    m = torch.arange(-j, j, dtype=torch.float64)
    raising = torch.diag(-torch.sqrt(j * (j + 1) - m * (m + 1)), diagonal=-1)
    m = torch.arange(-j + 1, j + 1, dtype=torch.float64)
    lowering = torch.diag(torch.sqrt(j * (j + 1) - m * (m - 1)), diagonal=1)
    m = torch.arange(-j, j + 1, dtype=torch.float64)
    su2 = torch.stack([
        (0.5 * (raising + lowering)).to(torch.complex128),
        torch.diag(1j * m.to(torch.complex128)),
        (-0.5j * (raising - lowering)).to(torch.complex128),
    ])
    q = torch.zeros((2 * l + 1, 2 * l + 1), dtype=torch.complex128)
    for mm in range(-l, 0):
        q[l + mm, l + abs(mm)] = 1 / 2**0.5
        q[l + mm, l - abs(mm)] = -1j / 2**0.5
    q[l, l] = 1
    for mm in range(1, l + 1):
        q[l + mm, l + abs(mm)] = (-1) ** mm / 2**0.5
        q[l + mm, l - abs(mm)] = 1j * (-1) ** mm / 2**0.5
    q = (-1j) ** l * q
    x = torch.conj(q.T) @ su2 @ q
    return torch.real(x)


@lru_cache(maxsize=None)
def _so3_generators_on(l: int, device: torch.device) -> torch.Tensor:
    """Device-resident copy, made once (a host-to-device copy is not graph-capturable)."""
    return _so3_generators(l).to(device)


def _matrix_x(a):
    c, s, o, z = a.cos(), a.sin(), torch.ones_like(a), torch.zeros_like(a)
    return torch.stack([torch.stack([o, z, z], -1), torch.stack([z, c, -s], -1), torch.stack([z, s, c], -1)], -2)


def _matrix_y(a):
    c, s, o, z = a.cos(), a.sin(), torch.ones_like(a), torch.zeros_like(a)
    return torch.stack([torch.stack([c, z, s], -1), torch.stack([z, o, z], -1), torch.stack([-s, z, c], -1)], -2)


def matrix_to_angles(r: torch.Tensor):
    """e3nn.o3.matrix_to_angles: R = Y(alpha) X(beta) Y(gamma)."""
    x = r[..., :, 1]  # R e_y
    x = torch.nn.functional.normalize(x, p=2, dim=-1).clamp(-1, 1)
    b = torch.acos(x[..., 1])
    a = torch.atan2(x[..., 0], x[..., 2])
    rr = (_matrix_y(a) @ _matrix_x(b) @ _matrix_y(torch.zeros_like(a))).transpose(-1, -2) @ r
    c = torch.atan2(rr[..., 0, 2], rr[..., 0, 0])
    return a, b, c


def _expm(a: torch.Tensor, squarings: int = 6, terms: int = 16) -> torch.Tensor:
    """exp of [..., n, n] float64 matrices by fixed scaling-and-squaring + Taylor. The generators
    are skew-symmetric with |eigenvalue| <= l <= 4 and angles < 2 pi, so ||a|| / 2^6 < 0.4 and 16
    terms are exact to float64 rounding; no data-dependent control flow (torch.matrix_exp reads
    norms back to the host), so it is safe inside a captured graph."""
    a = a / (2.0**squarings)
    eye = torch.eye(a.shape[-1], dtype=a.dtype, device=a.device).expand_as(a)
    out = eye.clone()
    for k in range(terms, 0, -1):  # Horner: I + a/1 (I + a/2 (I + ...))
        out = eye + (a @ out) / k
    for _ in range(squarings):
        out = out @ out
    return out


def wigner_d(l: int, alpha, beta, gamma) -> torch.Tensor:
    """e3nn.o3.wigner_D(l, alpha, beta, gamma) -> [..., 2l+1, 2l+1] (float64)."""
    gen = _so3_generators_on(l, alpha.device)
    a = (alpha.double() % (2 * math.pi))[..., None, None]
    b = (beta.double() % (2 * math.pi))[..., None, None]
    c = (gamma.double() % (2 * math.pi))[..., None, None]
    return _expm(a * gen[1]) @ _expm(b * gen[0]) @ _expm(c * gen[1])


def sh_rotation_matrix(rotations: torch.Tensor, d_sh: int) -> torch.Tensor:
    """Block-diagonal [..., d_sh, d_sh] real-SH rotation for each 3x3 rotation."""
    n_deg = math.isqrt(d_sh)
    a, b, c = matrix_to_angles(rotations.double())
    out = torch.zeros((*rotations.shape[:-2], d_sh, d_sh), dtype=torch.float64, device=rotations.device)
    for l in range(n_deg):
        out[..., l * l:(l + 1) ** 2, l * l:(l + 1) ** 2] = wigner_d(l, a, b, c)
    return out


@lru_cache(maxsize=None)
def x_basis_packed(device: torch.device) -> torch.Tensor:
    """The constant P^l = exp(-pi/2 X_z), l = 0..4, packed row-major (165 float64): e3nn's x
    rotation is P exp(t X_y) P^T. Device-resident, built once (kernel tsplat_sh_rotation_fwd)."""
    blocks = [_expm(-math.pi / 2 * _so3_generators(l)[2]).reshape(-1) for l in range(5)]
    return torch.cat(blocks).contiguous().to(device)


def rotate_sh(sh_coefficients: torch.Tensor, rotations: torch.Tensor) -> torch.Tensor:
    """sh [..., n] rotated by the per-camera rotation [..., 3, 3] (broadcast over pixels)."""
    n = sh_coefficients.shape[-1]
    d = sh_rotation_matrix(rotations, n).to(sh_coefficients.dtype)
    return torch.einsum("...ij,...j->...i", d, sh_coefficients)
