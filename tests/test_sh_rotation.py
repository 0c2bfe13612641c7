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
