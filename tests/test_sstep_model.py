"""The two-vectors-per-pass Lanczos model (tests/sstep_model.py) against the MGS
oracle (oracle/np_ref.py lanczos, eigen_krylov_complex.hpp:10-53): same T, same
f(L)u, orthonormal implicit basis; the shift is what keeps the Gram-derived norms
accurate.  CPU only, small grids."""
import numpy as np
import pytest

from oracle import np_ref
import sstep_model as sm


def _field(dim, n, seed=0):
    rng = np.random.default_rng(seed)
    L = 10.0
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    g = np.meshgrid(*([x] * dim), indexing="ij")
    r2 = sum(a * a for a in g)
    shape = (n,) * dim
    u = np.exp(-r2 / 4.0) * (1 + 0.1j) + 1e-3 * (rng.standard_normal(shape) + 1j * rng.standard_normal(shape))
    u = u.ravel()
    return u / np.sqrt(np.sum(np.abs(u) ** 2) * dx ** dim), dx


@pytest.mark.parametrize("dim,n,m", [(3, 12, 16), (2, 32, 16), (3, 10, 25), (2, 24, 10), (3, 10, 15)])
def test_tridiagonal_matches_mgs(dim, n, m):
    u, dx = _field(dim, n)
    nz = n if dim == 3 else 1
    ap = lambda v: np_ref.laplacian_apply(dim, n, n, nz, dx, dx, v)
    T, S, C, beta, G = sm.lanczos2(ap, u, m)
    _, Tr, br = np_ref.lanczos(ap, u, m)
    assert abs(beta - br) <= 1e-15 * br
    assert np.abs(T - np.real(Tr)).max() <= 1e-12 * np.abs(Tr).max()
    assert np.abs(C.conj().T @ G @ C - np.eye(m)).max() <= 1e-12


def test_shift_is_needed():
    u, dx = _field(3, 12)
    ap = lambda v: np_ref.laplacian_apply(3, 12, 12, 12, dx, dx, v)
    _, Tr, _ = np_ref.lanczos(ap, u, 16)
    err = {}
    for shift in (True, False):
        T, *_ = sm.lanczos2(ap, u, 16, shift=shift)
        err[shift] = np.abs(T - np.real(Tr)).max() / np.abs(Tr).max()
    assert err[True] < 1e-12 < err[False]


def test_nlse_trajectory_matches_oracle():
    u, dx = _field(3, 12)
    ref = np_ref.nlse_steps(3, 12, 12, 12, dx, dx, u, 1e-3, 8, 16)
    got, worst = sm.nlse_steps2(3, 12, dx, u, 1e-3, 8, 16)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 1e-12
    assert worst <= 1e-12


def test_g2_anisotropic_operator():
    n, m = 10, 25
    u, dx = _field(3, n, seed=3)
    x = np.linspace(-1, 1, n)
    g = np.meshgrid(x, x, x, indexing="ij")
    c = (1.0 + 0.3 * np.sin(2 * g[0]) * np.cos(g[1]) * np.cos(g[2])).ravel()
    A = np_ref.aniso_laplacian(3, n, n, n, dx, dx, c)
    ap = lambda v: A @ v
    T, S, C, beta, G = sm.lanczos2(ap, u, m)
    _, Tr, _ = np_ref.lanczos(ap, u, m)
    assert np.abs(T - np.real(Tr)).max() <= 1e-12 * np.abs(Tr).max()
    b2, _, _ = sm.krylov2(ap, u, 1j * 1e-3, m, np_ref.F_EXP)
    b1 = np_ref.krylov(ap, u, 1j * 1e-3, m, np_ref.F_EXP)
    assert np.linalg.norm(b2 - b1) / np.linalg.norm(b1) <= 1e-12


def test_sstep_schedule():
    assert sm.sstep_schedule(15) == [(0, 2), (2, 3), (5, 3), (8, 2), (10, 2), (12, 2)]
    assert sm.sstep_schedule(9) == [(0, 2), (2, 3), (5, 3)]
    assert sm.sstep_schedule(8) == [(0, 2), (2, 2), (4, 2), (6, 1)]
    assert sm.sstep_schedule(4) == [(0, 2), (2, 1)]
    assert sm.sstep_schedule(9, "all") == [(0, 2), (2, 3), (5, 3)]
    assert sm.sstep_schedule(8, "all") == [(0, 2), (2, 3), (5, 2)]
    assert sm.sstep_schedule(2) == [(0, 1)]
    for n in range(2, 33):  # every schedule stores exactly S_0..S_{n-1}
        s = sm.sstep_schedule(n)
        assert sum(ns for _, ns in s) == n - 1 and all(J + ns <= n - 1 for J, ns in s)
        # device rule: three-vector passes at J = 2, 5 only, two-vector ones at even J
        assert all((J in (2, 5)) if ns == 3 else J % 2 == 0 for J, ns in s)


@pytest.mark.parametrize("n,dx,m,p3", [(16, 20 / 511, 16, (2, 5)), (12, 20 / 511, 10, (2, 5)), (12, 0.5, 16, (2, 5)),
                                       (12, 20 / 511, 25, "all"), (12, 20 / 1023, 16, "all")])
def test_three_vector_passes_match_oracle(n, dx, m, p3):
    """Three new vectors per pass (radius-3 stencil of S_J) at the headline stiffness:
    the fused-tail result equals the MGS oracle's Krylov action."""
    rng = np.random.default_rng(5)
    ap = lambda v: np_ref.laplacian_apply(3, n, n, n, dx, dx, v)
    x = np.linspace(-1, 1, n)
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    u = (np.exp(-4 * (X * X + Y * Y + Z * Z)) * (1 + 0.2j) + 1e-3 * rng.standard_normal(X.shape)).ravel()
    ref = np_ref.krylov(ap, u, -1e-3j, m, np_ref.F_EXP_ABS)
    got, _ = sm.krylov_s_tail(ap, u, -1e-3j, m, np_ref.F_EXP_ABS, p3=p3)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 1e-12


@pytest.mark.parametrize("n,dx,kind", [(16, 20 / 511, "smooth"), (16, 20 / 511, "noise"), (12, 20 / 1023, "noise"),
                                       (12, 0.5, "noise")])
def test_four_vector_first_pass_matches_oracle(n, dx, kind):
    """A design study for the next pass form (DESIGN.md section 3 "Next"): the first pass
    writes four new vectors (a radius-4 stencil of S_0 alone, then two-vector passes from
    J = 4: 60 instead of 63 vector transfers at m = 16).  At the headline stiffness, and at
    twice it with white noise, the fused-tail action stays within 1e-12 of the MGS oracle."""
    rng = np.random.default_rng(5)
    ap = lambda v: np_ref.laplacian_apply(3, n, n, n, dx, dx, v)
    x = np.linspace(-1, 1, n)
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    amp = 1e-3 if kind == "smooth" else 1.0
    u = (np.exp(-4 * (X * X + Y * Y + Z * Z)) * (1 + 0.2j) + amp * rng.standard_normal(X.shape)).ravel()
    m = 16
    ref = np_ref.krylov(ap, u, -1e-3j, m, np_ref.F_EXP_ABS)
    sched = [(0, 4), (4, 2), (6, 2), (8, 2), (10, 2), (12, 2)]
    got, _ = sm.krylov_s_tail(ap, u, -1e-3j, m, np_ref.F_EXP_ABS, sched=sched)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 1e-12


@pytest.mark.parametrize("n,dx,kind,tol", [(16, 20 / 511, "smooth", 1e-13), (16, 20 / 511, "noise", 1e-13),
                                           (12, 20 / 1023, "noise", 5e-12), (12, 0.5, "noise", 1e-13)])
def test_four_vector_passes_at_every_j_match_oracle(n, dx, kind, tol):
    """The schedule a general four-vector pass would run: four new
    vectors at J = 0, 4, 8 and two at J = 12 -- 42 instead of 63 pass transfers at m = 16.
    At the headline stiffness the fused-tail action stays within 1e-13 of the MGS oracle;
    at twice it with white noise within 5e-12 (observed 2.2e-12; the two-vector schedule:
    4.6e-13), far inside the 1e-10 trajectory tolerance."""
    rng = np.random.default_rng(5)
    ap = lambda v: np_ref.laplacian_apply(3, n, n, n, dx, dx, v)
    x = np.linspace(-1, 1, n)
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    amp = 1e-3 if kind == "smooth" else 1.0
    u = (np.exp(-4 * (X * X + Y * Y + Z * Z)) * (1 + 0.2j) + amp * rng.standard_normal(X.shape)).ravel()
    m = 16
    ref = np_ref.krylov(ap, u, -1e-3j, m, np_ref.F_EXP_ABS)
    sched = [(0, 4), (4, 4), (8, 4), (12, 2)]
    assert sum(J + ns + 1 for J, ns in sched) == 42  # reads S_0..S_J, writes ns
    got, _ = sm.krylov_s_tail(ap, u, -1e-3j, m, np_ref.F_EXP_ABS, sched=sched)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= tol
