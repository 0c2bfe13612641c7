"""e3nn-free Wigner-D (transplat_amd/misc/sh_rotation.py): the only in-repo pin of the reference
(fast_sh_rotation.py:56-60) concerns l = 1 and is not asserted by its own script; what is checked
here is the construction itself: D^1 = R in e3nn's (x, y, z) real basis, orthogonality, the
homomorphism D(R1 R2) = D(R1) D(R2), angle round trip, and the graph-safe expm vs torch's."""
import pytest
import torch
from scipy.spatial.transform import Rotation as Rs

from transplat_amd.misc import sh_rotation as shr


def rots(n, seed):
    return torch.tensor(Rs.random(n, random_state=seed).as_matrix())


def test_d1_equals_rotation():
    r = rots(8, 0)
    d = shr.wigner_d(1, *shr.matrix_to_angles(r))
    assert (d - r).abs().max() < 1e-12


@pytest.mark.parametrize("l", [0, 1, 2, 3, 4])
def test_orthogonal_and_homomorphism(l):
    r1, r2 = rots(6, 1), rots(6, 2)
    a = shr.wigner_d(l, *shr.matrix_to_angles(r1))
    b = shr.wigner_d(l, *shr.matrix_to_angles(r2))
    c = shr.wigner_d(l, *shr.matrix_to_angles(r1 @ r2))
    eye = torch.eye(2 * l + 1, dtype=torch.float64)
    assert (a @ a.transpose(-1, -2) - eye).abs().max() < 1e-12
    assert (a @ b - c).abs().max() < 1e-12


def test_expm_matches_torch():
    for l in range(5):
        g = shr._so3_generators(l)
        for ang in (0.1, 2.0, 6.28):
            assert (shr._expm(ang * g[1]) - torch.matrix_exp(ang * g[1])).abs().max() < 1e-12


def test_block_diagonal_rotation_identity():
    d = shr.sh_rotation_matrix(torch.eye(3, dtype=torch.float64)[None], 25)
    assert (d[0] - torch.eye(25, dtype=torch.float64)).abs().max() < 1e-12


def _factored(r, l):
    """The factorisation tsplat_sh_rotation_fwd evaluates: D^l = Z(a) P Z(b) P^T Z(c) with
    Z(t) = exp(t X_y) written out (cos(|m| t) diagonal, +-sin(|m| t) anti-diagonal) and
    P = exp(-pi/2 X_z)."""
    import math

    a, b, c = shr.matrix_to_angles(r)
    n = 2 * l + 1

    def z(t):
        out = torch.zeros((*t.shape, n, n), dtype=torch.float64)
        for i in range(n):
            m = i - l
            out[..., i, i] = torch.cos(abs(m) * t)
            if m != 0:
                out[..., i, 2 * l - i] = torch.sin(abs(m) * t) * (1 if m < 0 else -1)
        return out

    p = torch.matrix_exp(-math.pi / 2 * shr._so3_generators(l)[2])
    return z(a) @ p @ z(b) @ p.T @ z(c)


@pytest.mark.parametrize("l", [1, 2, 3, 4])
def test_kernel_factorisation_matches_expm_form(l):
    r = rots(16, 3)
    assert (_factored(r, l) - shr.wigner_d(l, *shr.matrix_to_angles(r))).abs().max() < 1e-12


def test_x_basis_packed_layout():
    p = shr.x_basis_packed(torch.device("cpu"))
    assert p.shape == (165,) and p.dtype == torch.float64
    assert (p[1:10].reshape(3, 3) @ p[1:10].reshape(3, 3).T - torch.eye(3, dtype=torch.float64)).abs().max() < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("d_sh", [1, 4, 9, 16, 25])
def test_sh_rotation_kernel(device, d_sh):
    from transplat_amd import kernels

    r = rots(64, 4)
    r[0] = torch.eye(3, dtype=torch.float64)  # gimbal-aligned special cases
    r[1] = torch.diag(torch.tensor([-1.0, 1.0, -1.0], dtype=torch.float64))
    ref = shr.sh_rotation_matrix(r.float().double(), d_sh)
    out = kernels.sh_rotation(r.float().to(device), d_sh).cpu().double()
    assert (out - ref).abs().max().item() < 2e-6
