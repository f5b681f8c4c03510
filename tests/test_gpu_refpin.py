"""GPU against fixtures computed by the reference's own executable Python
(tests/golden/make_ref_fixtures.py): the Krylov action built from the V and T of
LanczosStepTorch (nlsolvers/fusing_kernels.py:8-45) and the 2D Neumann BC of
neumann_bc (bc_update_kernel_fusion.py:18-27).  No oracle in the loop: the
reference's numbers directly.

Tolerances: Krylov action <= 1e-12 (as every GPU action test), BC bit-exact.
"""
import os

import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_LANCZOS = ["ref_lanczos_2d_smooth", "ref_lanczos_2d_noise", "ref_lanczos_3d_smooth",
               "ref_lanczos_3d_noise"]


def ref_action(d, m, t):
    T = d[f"T{m}"]
    H = np.tril(T, -1) + np.tril(T, -1).conj().T + np.diag(T.diagonal().real)
    lam, Q = np.linalg.eigh(H)
    return float(d["beta0"]) * (d["V16"][:m].T @ (Q @ (np.exp(t * np.abs(lam)) * Q[0].conj())))


@pytest.mark.parametrize("pass2", ["1", "0"])
@pytest.mark.parametrize("name", REF_LANCZOS)
@pytest.mark.parametrize("m", [10, 16])
def test_gpu_action_matches_reference_lanczos(monkeypatch, pass2, name, m):
    """G1 exp(t|lambda|) action on the GPU (two-vector s-step passes, and the one-vector
    passes) == beta0 V Q f(Lambda) Q^H e1 from the reference's own V, T."""
    monkeypatch.setenv("NLS_PASS2", pass2)
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    dim, n, dx = int(d["dim"]), int(d["n"]), float(d["dx"])
    with nls_amd.Solver(dim, n, n, n, dx, dx, m=m) as s:
        for t in (-1e-3j, -1e-2j):
            got = s.krylov_apply(d["u"], t, nls_amd.F_EXP_ABS)
            assert rel_l2(got, ref_action(d, m, t)) <= 1e-12


def test_gpu_neumann_bc_matches_reference():
    """nls_apply_bc (k_neumann_bc) == the reference's neumann_bc, bit for bit, on a
    square and a non-square complex field (tensor axis 0 = our rows, ny)."""
    d = np.load(os.path.join(GOLD, "ref_bc2d.npz"))
    for a, b in ((24, 24), (9, 13)):
        with nls_amd.Solver(2, b, a, 1, 0.5, 0.5, equation=nls_amd.NLSE_G2, m=4) as s:
            s.set_coefficients(np.ones(a * b), np.ones(a * b))
            s.set_field(d[f"uc_{a}x{b}"].ravel())
            s.apply_bc()
            assert np.array_equal(s.get_field().reshape(a, b), d[f"bc_c_{a}x{b}"])


def test_gpu_neumann_bc_real_matches_reference():
    """The real-field BC of the Klein-Gordon drivers (k_neumann_bc_r) == neumann_bc on f64."""
    d = np.load(os.path.join(GOLD, "ref_bc2d.npz"))
    for a, b in ((24, 24), (9, 13)):
        with nls_amd.Solver(2, b, a, 1, 0.5, 0.5, equation=nls_amd.KG_GAUTSCHI, m=4) as s:
            s.set_coefficients(np.ones(a * b), np.ones(a * b))
            u = d[f"ur_{a}x{b}"].ravel()
            s.set_sg_state(u, u)
            s.apply_bc()
            assert np.array_equal(s.get_field().reshape(a, b), d[f"bc_r_{a}x{b}"])
