"""CPU tests of the oracle (test infrastructure) -- pins it before it is trusted.

1. Operator: the matrix-free restatement equals a literal transcription of the
   reference triplet builders (laplacians.hpp:10-105), entry for entry, and
   shows the quirks the survey measured (3D y-wrap, non-NSD 3D operator).
2. Known-answer test from the reference's own published artefact
   (nlsolvers/scipy-test/data/_comparison_without_lanczos_check.png, setup
   nlsolvers/host/drivers/test_scipy_matfunc.cpp:41-95 and
   nlsolvers/scipy-test/check_krylov_compute.py:41-49): Krylov exp action vs
   scipy.sparse.linalg.expm_multiply, 3D 50^3, L=2, t=1e-2.
3. Two independent restatements (C oracle, numpy twin with eigh) agree.
4. Golden fixtures (tests/golden/make_golden.py) are reproduced.
5. Fixtures computed by the REFERENCE'S OWN executable Python
   (tests/golden/make_ref_fixtures.py: LanczosStepTorch, fusing_kernels.py:8-45,
   and neumann_bc, bc_update_kernel_fusion.py:18-27) pin the oracle's Lanczos
   recurrence (V, T, beta), its Krylov action and its 2D Neumann BC.
"""
import os

import numpy as np
import pytest
import scipy.sparse.linalg as spla

import np_ref
import oracle_py as O
from conftest import rel_l2

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("dim,n", [(2, 2), (2, 5), (2, 12), (3, 2), (3, 4), (3, 7)])
def test_operator_equals_triplet_builder(dim, n):
    dx = 0.37
    A = np_ref.laplacian_triplets(dim, n, dx)
    N = A.shape[0]
    g = O.grid(dim, n, n, n, dx, dx)
    rng = np.random.default_rng(n)
    for _ in range(2):
        x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        ref = A @ x
        assert np.array_equal(O.laplacian_c(g, x), ref) or rel_l2(O.laplacian_c(g, x), ref) < 1e-15
        assert rel_l2(O.laplacian_r(g, x.real), A @ x.real) < 1e-15
        assert rel_l2(np_ref.laplacian_apply(dim, n, n, n, dx, dx, x), ref) < 1e-15
    # exact matrix reconstruction from the matrix-free apply (unit vectors)
    if N <= 400:
        M = np.column_stack([O.laplacian_r(g, np.eye(N)[:, k]) for k in range(N)])
        assert np.array_equal(M, A.toarray())


def test_operator_quirks():
    n = 8
    dx = 1.0
    A = np_ref.laplacian_triplets(3, n, dx).toarray()
    assert np.array_equal(A, A.T)
    # 3D y-wrap couplings (i, n-1, k) <-> (i, 0, k+1) for k < n-1: n*(n-1) of them
    wrap = 0
    for k in range(n - 1):
        for i in range(n):
            p = k * n * n + (n - 1) * n + i
            q = (k + 1) * n * n + 0 * n + i
            wrap += A[p, q] != 0
    assert wrap == n * (n - 1)
    # the 3D operator is not negative semi-definite: max eig +0.299/dx^2 at n=8
    ev = np.linalg.eigvalsh(A)
    assert 0.29 < ev.max() < 0.31
    # boundary diagonals -5 (3D) / -3 (2D), not minus the neighbour count
    assert A[0, 0] == -5.0 and A[n * n * (n // 2) + n * (n // 2) + n // 2, n * n * (n // 2) + n * (n // 2) + n // 2] == -6.0
    A2 = np_ref.laplacian_triplets(2, n, dx).toarray()
    assert A2[0, 0] == -3.0 and np.linalg.eigvalsh(A2).max() < 0


def _kat_setup():
    n, L, t = 50, 2.0, 1e-2
    dx = 2 * L / n
    A = np_ref.aniso_laplacian_3d(n, dx, np.ones(n ** 3))
    u0 = np_ref.centered_gaussian_3d(n, L, L / 5)
    return A, u0, t


def test_scipy_kat():
    """Published accuracy (plot): real m=10 ~5e-10, m>=20 ~2e-15; complex m=10 ~1.2e-9,
    m>=20 ~3e-13.  The oracle must land on those values (G2 exp(t*lambda) convention)."""
    A, u0, t = _kat_setup()
    ys = spla.expm_multiply(A, u0, start=0, stop=t, endpoint=True, num=2)[-1]
    yc = spla.expm_multiply(1j * A.astype(np.complex128), u0.astype(np.complex128),
                            start=0, stop=t, endpoint=True, num=2)[-1]
    er = {m: rel_l2(O.krylov_csr(A, u0, t, m, O_F_EXP), ys) for m in (10, 20, 30)}
    ec = {m: rel_l2(O.krylov_csr(A, u0.astype(complex), 1j * t, m, O_F_EXP), yc) for m in (10, 20, 30)}
    assert 3e-10 < er[10] < 9e-10, er
    assert er[20] < 1e-13 and er[30] < 1e-13, er
    assert 7e-10 < ec[10] < 2e-9, ec
    assert 5e-14 < ec[20] < 1e-12 and ec[30] < 1e-12, ec


O_F_EXP = 1


@pytest.mark.parametrize("dim,n", [(2, 20), (3, 8)])
def test_oracle_matches_numpy_twin(dim, n):
    L = 5.0
    dx = 2 * L / (n - 1)
    g = O.grid(dim, n, n, n, dx, dx)
    rng = np.random.default_rng(9)
    N = n ** dim
    u = np.exp(-np.linspace(-2, 2, N) ** 2) + 1e-2 * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
    ap = lambda v: np_ref.laplacian_apply(dim, n, n, n, dx, dx, v)
    for m in (1, 2, 10, 16):
        a = O.krylov_c(g, u, -1e-3j, m, 0)
        b = np_ref.krylov(ap, u, -1e-3j, m, 0)
        assert rel_l2(a, b) < 1e-13
    for f in (2, 3, 4, 5, 6):
        a = O.krylov_r(g, u.real, 1e-2, 10, f)
        b = np_ref.krylov(ap, u.real, 1e-2, 10, f)
        assert rel_l2(a, b) < 1e-12
    a = O.nlse_steps(g, u, 1e-3, 5, 10)
    b = np_ref.nlse_steps(dim, n, n, n, dx, dx, u, 1e-3, 5, 10)
    assert rel_l2(a, b) < 1e-13
    a = O.nlse_steps(g, u, 1e-3, 5, 10, nonlin=1)
    b = np_ref.nlse_steps(dim, n, n, n, dx, dx, u, 1e-3, 5, 10, nonlin=1)
    assert rel_l2(a, b) < 1e-13


def test_oracle_structural_properties():
    """exp of a Hermitian T is unitary and the nonlinear phase has unit modulus:
    the cubic SS2 step conserves the discrete L2 norm."""
    n, L = 24, 10.0
    dx = 2 * L / (n - 1)
    g = O.grid(2, n, n, 1, dx, dx)
    rng = np.random.default_rng(0)
    u = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
    out = O.nlse_steps(g, u, 1e-3, 10, 16)
    assert abs(np.linalg.norm(out) / np.linalg.norm(u) - 1) < 1e-13
    # m = 1: T = [0] so exp(T) = 1 and the linear part is the identity
    out1 = O.krylov_c(g, u, -1e-3j, 1, 0)
    assert rel_l2(out1, u) < 1e-15


def test_reference_breakdown_semantics():
    """The Eigen path divides by beta = 0 (eigen_krylov_complex.hpp:20,47): NaN.
    The device library follows the device guard instead (tests/test_gpu_parity.py)."""
    g = O.grid(2, 8, 8, 1, 1.0, 1.0)
    with np.errstate(all="ignore"):
        out = O.krylov_c(g, np.zeros(64, complex), -1e-3j, 4, 0)
    assert np.all(np.isnan(out))


@pytest.mark.parametrize("name", ["nlse2d", "cq2d", "nlse3d"])
def test_golden_nlse(name):
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    n, dim = int(d["n"]), int(d["dim"])
    g = O.grid(dim, n, n, n, float(d["dx"]), float(d["dx"]))
    out = O.nlse_steps(g, d["u0"], float(d["dt"]), int(d["steps"]), int(d["m"]), nonlin=int(d["nonlin"]))
    assert rel_l2(out, d["u"]) < 1e-13
    tw = np_ref.nlse_steps(dim, n, n, n, float(d["dx"]), float(d["dx"]), d["u0"], float(d["dt"]),
                           int(d["steps"]), int(d["m"]), nonlin=int(d["nonlin"]))
    assert rel_l2(tw, d["u"]) < 1e-12


def test_golden_sg():
    d = np.load(os.path.join(GOLD, "sg2d.npz"))
    n = int(d["n"])
    g = O.grid(2, n, n, 1, float(d["dx"]), float(d["dx"]))
    u, up = O.sg_steps(g, d["u0"], d["u_past0"], d["mfield"], float(d["dt"]), int(d["steps"]), int(d["m"]))
    assert rel_l2(u, d["u"]) < 1e-13 and rel_l2(up, d["u_past"]) < 1e-13


def test_golden_krylov_functions():
    d = np.load(os.path.join(GOLD, "krylov3d.npz"))
    n, m = int(d["n"]), int(d["m"])
    g = O.grid(3, n, n, n, float(d["dx"]), float(d["dx"]))
    for f in (2, 3, 4, 5, 6):
        assert rel_l2(O.krylov_r(g, d["ur"], 1e-2, m, f), d[f"r_f{f}"]) < 1e-13
    assert rel_l2(O.krylov_c(g, d["uc"], -1e-2j, m, 0), d["c_f0"]) < 1e-13
    assert rel_l2(O.krylov_c(g, d["uc"], 1e-2j, m, 1), d["c_f1"]) < 1e-13
    assert rel_l2(O.laplacian_c(g, d["uc"]), d["lap"]) < 1e-15


# ---------------------------------------------------------------------------
# G2 (nlsolvers/): anisotropic operator, exp(t*lambda) stepper, Neumann copy BC


@pytest.mark.parametrize("dim,nx,ny,nz", [(2, 3, 3, 1), (2, 9, 7, 1), (3, 3, 3, 3), (3, 6, 5, 4)])
def test_aniso_operator_equals_builder(dim, nx, ny, nz):
    """Matrix-free G2 operator == the triplet builder
    (nlsolvers/common/include/laplacians.hpp:54-103, 158-218), entry for entry."""
    N = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(N)
    c = rng.uniform(0.2, 3.0, N)
    A = np_ref.aniso_laplacian(dim, nx, ny, nz, 0.31, 0.29, c).toarray()
    g = O.grid(dim, nx, ny, nz, 0.31, 0.29)
    M = np.stack([O.laplacian_aniso_c(g, c, np.eye(N)[k]) for k in range(N)], axis=1)
    assert np.allclose(M, A, rtol=1e-15, atol=1e-15)
    assert np.array_equal(A, A.T)
    # the diagonal is minus the row sum of the couplings: constants are in the kernel
    assert np.allclose(A.sum(axis=1), 0.0, atol=1e-12)


def test_aniso_quirks():
    """c == 1 is NOT the isotropic operator (diagonal = -#couplings), and the 3D
    builder keeps the flat-index y-wrap (i, ny-1, k) <-> (i, 0, k+1)."""
    n = 5
    Aa = np_ref.aniso_laplacian(3, n, n, n, 1.0, 1.0, np.ones(n ** 3)).toarray()
    Ai = np_ref.laplacian_triplets(3, n, 1.0).toarray()
    off = ~np.eye(n ** 3, dtype=bool)
    assert np.array_equal(Aa[off], Ai[off])
    assert not np.array_equal(np.diag(Aa), np.diag(Ai))
    p = (0 * n + (n - 1)) * n + 2          # (i=2, j=n-1, k=0)
    q = (1 * n + 0) * n + 2                # (i=2, j=0, k=1)
    assert Aa[p, q] == 1.0


def test_scipy_kat_stencil_operator():
    """The published KAT again, now through the matrix-free G2 operator the
    device kernels restate (c == 1, full 50^3 grid) -- same error levels."""
    A, u0, t = _kat_setup()
    n, L = 50, 2.0
    g = O.grid(3, n, n, n, 2 * L / n, 2 * L / n)
    ones = np.ones(n ** 3)
    yc = spla.expm_multiply(1j * A.astype(np.complex128), u0.astype(np.complex128),
                            start=0, stop=t, endpoint=True, num=2)[-1]
    ec = {m: rel_l2(O.krylov_aniso_c(g, ones, u0, 1j * t, m, O_F_EXP), yc) for m in (10, 20)}
    assert 7e-10 < ec[10] < 2e-9, ec
    assert 5e-14 < ec[20] < 1e-12, ec


@pytest.mark.parametrize("dim,nx,ny,nz", [(2, 3, 3, 1), (2, 8, 11, 1), (3, 3, 4, 5), (3, 7, 6, 5)])
def test_neumann_bc(dim, nx, ny, nz):
    """The reference's copy sequence (boundaries.cuh:10-81) == the clamp gather
    the device kernel implements; interior untouched; idempotent."""
    N = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(N)
    u = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    g = O.grid(dim, nx, ny, nz, 1.0, 1.0)
    b = O.neumann_bc(g, u)
    assert np.array_equal(b, np_ref.neumann_bc(dim, nx, ny, nz, u))
    assert np.array_equal(O.neumann_bc(g, b), b)
    shp = (ny, nx) if dim == 2 else (nz, ny, nx)
    inner = tuple(slice(1, s - 1) for s in shp)
    assert np.array_equal(b.reshape(shp)[inner], u.reshape(shp)[inner])


@pytest.mark.parametrize("dim,n,m", [(2, 16, 20), (3, 8, 25)])
def test_g2_oracle_matches_numpy_twin(dim, n, m):
    rng = np.random.default_rng(dim)
    N = n ** dim
    dx = 0.5
    c = rng.uniform(0.5, 2.0, N)
    mf = rng.uniform(-1.0, 2.0, N)
    u = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    g = O.grid(dim, n, n, n, dx, dx)
    for bc in (False, True):
        a = O.nlse_g2_steps(g, c, mf, u, 1e-3, 4, m, bc=bc)
        b = np_ref.nlse_g2_steps(dim, n, n, n, dx, dx, c, mf, u, 1e-3, 4, m, bc=bc)
        assert rel_l2(a, b) < 1e-12
    # no BC, the G2 step is unitary too (Hermitian T, unit-modulus phase)
    a = O.nlse_g2_steps(g, c, mf, u, 1e-3, 4, m, bc=False)
    assert abs(np.linalg.norm(a) / np.linalg.norm(u) - 1) < 1e-12


@pytest.mark.parametrize("name", ["g2_3d", "g2_2d"])
def test_golden_g2(name):
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    n, dim = int(d["n"]), int(d["dim"])
    g = O.grid(dim, n, n, n, float(d["dx"]), float(d["dx"]))
    out = O.nlse_g2_steps(g, d["c"], d["mfield"], d["u0"], float(d["dt"]), int(d["steps"]), int(d["m"]))
    assert rel_l2(out, d["u"]) < 1e-13


@pytest.mark.parametrize("dim,n,m", [(2, 16, 15), (3, 8, 15)])
def test_cq_g2_oracle_matches_numpy_twin(dim, n, m):
    """G2 cubic-quintic (nlse_cubic_quintic_dev.hpp:79-95), two restatements; in 2D the
    twin uses the triplet builder (laplacians.hpp:10-52), in 3D the stencil."""
    rng = np.random.default_rng(60 + dim)
    N = n ** dim
    mf = rng.uniform(0.5, 1.5, N)
    u = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    g = O.grid(dim, n, n, n, 0.5, 0.5)
    for bc in (False, True):
        a = O.nlse_cq_g2_steps(g, mf, u, 1e-3, 4, m, 1.0, -0.5, bc=bc)
        b = np_ref.nlse_cq_g2_steps(dim, n, n, n, 0.5, 0.5, mf, u, 1e-3, 4, m, 1.0, -0.5, bc=bc)
        assert rel_l2(a, b) < 1e-12
    # real sigmas: the phase has unit modulus and T is Hermitian, so no BC = unitary
    a = O.nlse_cq_g2_steps(g, mf, u, 1e-3, 4, m, 1.0, -0.5, bc=False)
    assert abs(np.linalg.norm(a) / np.linalg.norm(u) - 1) < 1e-12
    # rho = m (s1 d + s2 d^2): m = 2 with (s1, s2) is m = 1 with (2 s1, 2 s2)
    a = O.nlse_cq_g2_steps(g, 2.0 * np.ones(N), u, 1e-3, 2, m, 1.0, -0.5, bc=True)
    c = O.nlse_cq_g2_steps(g, np.ones(N), u, 1e-3, 2, m, 2.0, -1.0, bc=True)
    assert rel_l2(a, c) < 1e-14


def test_golden_cq_g2():
    d = np.load(os.path.join(GOLD, "cq_g2_2d.npz"))
    n = int(d["n"])
    g = O.grid(2, n, n, 1, float(d["dx"]), float(d["dx"]))
    out = O.nlse_cq_g2_steps(g, d["mfield"], d["u0"], float(d["dt"]), int(d["steps"]), int(d["m"]),
                             float(d["s1"]), float(d["s2"]), bc=True)
    assert rel_l2(out, d["u"]) < 1e-13


@pytest.mark.parametrize("dim,n,m", [(2, 14, 25), (3, 7, 15)])
def test_sewi_oracle_matches_numpy_twin(dim, n, m):
    """G2 sEWI (nlsolvers/device/include/nlse_dev.hpp:205-238), two restatements."""
    rng = np.random.default_rng(11 + dim)
    N = n ** dim
    c = rng.uniform(0.5, 2.0, N)
    mf = rng.uniform(0.5, 1.5, N)
    u = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    g = O.grid(dim, n, n, n, 0.6, 0.6)
    a, ap = O.nlse_sewi_steps(g, c, mf, u, None, 1e-3, 1, 4, m, bc=True)
    b, bp = np_ref.nlse_sewi_steps(dim, n, n, n, 0.6, 0.6, c, mf, u, None, 1e-3, 1, 4, m, bc=True)
    assert rel_l2(a, b) < 1e-12 and rel_l2(ap, bp) < 1e-12
    # resuming at step 3 with the state after step 2 is the same trajectory
    s2, s2p = O.nlse_sewi_steps(g, c, mf, u, None, 1e-3, 1, 2, m, bc=True)
    r, rp = O.nlse_sewi_steps(g, c, mf, s2, s2p, 1e-3, 3, 2, m, bc=True)
    assert np.array_equal(r, a) and np.array_equal(rp, ap)


def test_sinc_function_convention():
    """G2 "sinc" is sinc(t*lambda) with no |.| or sqrt (matfunc_complex.hpp:293-300):
    on a 1-D invariant subspace (an eigenvector of L) the action is the scalar map."""
    n = 6
    g = O.grid(2, n, n, 1, 1.0, 1.0)
    ones = np.ones(n * n)
    # constants are in the kernel of div(c grad): lambda = 0 -> sinc = 1
    v = np.ones(n * n, complex)
    assert rel_l2(O.krylov_aniso_c(g, ones, v, 0.3, 4, 7), v) < 1e-14
    A = np_ref.aniso_laplacian(2, n, n, 1, 1.0, 1.0, ones).toarray()
    lam, Q = np.linalg.eigh(A)
    q = Q[:, 3].astype(complex)
    t = 0.37
    want = np.sin(t * lam[3]) / (t * lam[3]) * q
    assert rel_l2(O.krylov_aniso_c(g, ones, q, t, 3, 7), want) < 1e-12


def test_golden_sewi():
    d = np.load(os.path.join(GOLD, "sewi_3d.npz"))
    n = int(d["n"])
    g = O.grid(3, n, n, n, float(d["dx"]), float(d["dx"]))
    u, up = O.nlse_sewi_steps(g, d["c"], d["mfield"], d["u0"], None, float(d["dt"]), 1, int(d["steps"]),
                              int(d["m"]))
    assert rel_l2(u, d["u"]) < 1e-13 and rel_l2(up, d["u_prev"]) < 1e-13


@pytest.mark.parametrize("dim,n", [(2, 14), (3, 7)])
def test_kg_oracle_matches_numpy_twin(dim, n):
    """G2 Klein-Gordon Gautschi (kg_single.cuh:49-86) on -div(c grad), two restatements;
    the velocity is a difference quotient, so it carries an extra 1/dt."""
    rng = np.random.default_rng(21 + dim)
    N = n ** dim
    c = rng.uniform(0.5, 2.0, N)
    mf = rng.uniform(0.5, 1.5, N)
    u = rng.standard_normal(N)
    dt = 1e-2
    up = u - dt * 0.1 * rng.standard_normal(N)
    g = O.grid(dim, n, n, n, 0.6, 0.6)
    a = O.kg_steps(g, c, mf, u, up, dt, 4, 10, bc=True)
    b = np_ref.kg_steps(dim, n, n, n, 0.6, 0.6, c, mf, u, up, dt, 4, 10, bc=True)
    assert rel_l2(a[0], b[0]) < 1e-12 and rel_l2(a[1], b[1]) < 1e-12 and rel_l2(a[2], b[2]) < 1e-10


def test_kg_operator_sign_is_immaterial():
    """The KG drivers pass -div(c grad); cos / sinc^2 of t sqrt|lambda| are even in the
    operator sign (T -> -S T S), so +L gives the same action up to rounding."""
    n = 9
    g = O.grid(2, n, n, 1, 0.5, 0.5)
    rng = np.random.default_rng(4)
    c = rng.uniform(0.5, 2.0, n * n)
    u = rng.standard_normal(n * n)
    A = np_ref.aniso_laplacian(2, n, n, 1, 0.5, 0.5, c)
    for f in (np_ref.F_COS_SQRT, np_ref.F_SINC2_SQRT):
        assert rel_l2(np_ref.krylov(lambda x: A @ x, u, 0.05, 8, f),
                      np_ref.krylov(lambda x: -(A @ x), u, 0.05, 8, f)) < 1e-13


def test_golden_kg():
    d = np.load(os.path.join(GOLD, "kg_3d.npz"))
    n, dt = int(d["n"]), float(d["dt"])
    g = O.grid(3, n, n, n, float(d["dx"]), float(d["dx"]))
    u, up, v = O.kg_steps(g, d["c"], d["mfield"], d["u0"], d["u0"] - dt * d["v0"], dt, int(d["steps"]),
                          int(d["m"]))
    assert rel_l2(u, d["u"]) < 1e-13 and rel_l2(up, d["u_past"]) < 1e-13 and rel_l2(v, d["v"]) < 1e-11


# ---- G2 Gautschi family: sg_single / sg_double / sg_hyperbolic / phi4 -------------

@pytest.mark.parametrize("kind", sorted(O.GG_KINDS.values()))
@pytest.mark.parametrize("dim,n", [(2, 15), (3, 8)])
def test_gautschi_g2_oracle_matches_numpy_twin(kind, dim, n):
    """Phi4Solver / SGE{,Double,Hyperbolic}Solver::step (phi4_single.cuh:33-47,
    sg_single.cuh:33-47, sg_double.cuh:34-48, sg_hyperbolic.cuh:33-47) + apply_bc,
    two restatements (C: cyclic Jacobi, numpy: LAPACK eigh)."""
    rng = np.random.default_rng(61 + kind + dim)
    N = n ** dim
    u = rng.standard_normal(N)
    dt = 1e-2
    up = u - dt * 0.1 * rng.standard_normal(N)
    mf = rng.uniform(0.5, 1.5, N)
    g = O.grid(dim, n, n, n, 0.5, 0.5)
    a = O.gautschi_g2_steps(g, kind, u, up, mf, dt, 4, 10, bc=True)
    b = np_ref.gautschi_g2_steps(dim, n, n, n, 0.5, 0.5, kind, u, up, mf, dt, 4, 10, bc=True)
    assert rel_l2(a[0], b[0]) < 1e-12 and rel_l2(a[1], b[1]) < 1e-12


def test_gautschi_g2_family_differs_only_in_force():
    """At small amplitude all four forces are ~ u to first order (sin, sinh, u + u^3,
    and the double sine ~ 1.5 u): the trajectories of sin / sinh / phi4 agree to
    O(u^3) and differ in the expected direction of the cubic term."""
    n = 16
    rng = np.random.default_rng(3)
    u = 1e-3 * rng.standard_normal(n * n)
    mf = np.ones(n * n)
    g = O.grid(2, n, n, 1, 0.4, 0.4)
    outs = {k: O.gautschi_g2_steps(g, v, u, u, mf, 1e-2, 5, 10)[0] for k, v in O.GG_KINDS.items()}
    assert rel_l2(outs["sg"], outs["phi4"]) < 1e-5
    assert rel_l2(outs["sg"], outs["sg_hyperbolic"]) < 1e-5
    assert rel_l2(outs["sg"], outs["sg_double"]) > 1e-8  # 1.5x the linear force


def test_gautschi_g2_uses_full_sinc2_argument():
    """The G2 device family filters g with sinc^2(t sqrt|lambda|) (matfunc_real.hpp:212-219),
    not the G1 CPU path's sinc^2(t/2 sqrt|lambda|) (eigen_krylov_real.hpp:172-201): with the
    sine force, m = -1 and no BC it must differ from oracle_sg_steps at O(dt^4 ||L||)."""
    n = 16
    x = np.linspace(-3, 3, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    u = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y)))).ravel()
    g = O.grid(2, n, n, 1, 0.4, 0.4)
    a, _ = O.gautschi_g2_steps(g, 0, u, u, np.ones(n * n), 1e-2, 3, 10, bc=False)
    b, _ = O.sg_steps(g, u, u, -np.ones(n * n), 1e-2, 3, 10)
    assert 1e-12 < rel_l2(a, b) < 1e-3


def test_golden_gautschi_g2():
    d = np.load(os.path.join(GOLD, "gautschi_g2.npz"))
    n, dt = int(d["n"]), float(d["dt"])
    g = O.grid(2, n, n, 1, float(d["dx"]), float(d["dx"]))
    for kname, kind in O.GG_KINDS.items():
        u, up = O.gautschi_g2_steps(g, kind, d["u0"], d["u0"] - dt * d["v0"], d["mfield"], dt,
                                    int(d["steps"]), int(d["m"]))
        assert rel_l2(u, d[f"u_{kname}"]) < 1e-13 and rel_l2(up, d[f"u_past_{kname}"]) < 1e-13


# ---- pins from the reference's own executable code (tests/golden/make_ref_fixtures.py) ----
# Measured differences (oracle MGS vs the reference's CGS step, fresh-dot T(j-1, j)):
# T 1e-15 .. 4.3e-15 of max|T|, beta <= 1e-15, V <= 9e-15 per vector, at every spacing
# (the Lanczos basis of c L is that of L: the stiffness enters the recurrence only through
# rounding).  The bounds below are ~25x that: a change of recurrence (a missing
# re-orthogonalisation term, a wrong T write, another normalisation) moves these by orders
# of magnitude.  The Krylov ACTION inherits the eigenvalues' relative rounding times the
# argument of f: its error is ~ eps (1 + kappa) with kappa = |t| rho(T) (exp, sinc of
# t lambda) or |t| sqrt(rho(T)) (the t sqrt|lambda| functions) -- observed at most
# 38 eps (1 + kappa) over every fixture, spacing and function (sinc^2 at C4's spacing,
# kappa = 38); TOL_REF_ACT_K = 200 eps.
REF_COMPLEX = ["ref_lanczos_2d_smooth", "ref_lanczos_2d_noise", "ref_lanczos_3d_smooth",
               "ref_lanczos_3d_noise"]
REF_REAL = [f"{n}_real" for n in REF_COMPLEX]
# the same noise fields at the BASELINE workloads' spacings: hl = 20/511 (3D 512^3),
# c2 = 20/4095 (2D 4096^2), c4 = 6/8191 (sine-Gordon 8192^2)
REF_STIFF = [f"ref_lanczos_{d}d_noise{r}_{s}" for d in (2, 3) for r in ("", "_real")
             for s in ("hl", "c2", "c4")]
REF_LANCZOS = REF_COMPLEX + REF_REAL + REF_STIFF
TOL_REF_T, TOL_REF_V = 1e-13, 2.5e-13
TOL_REF_ACT_K = 200 * 2.22e-16
REAL_FUNCS = (2, 3, 4, 5, 6)  # cos, sinc, sinc^2, id of t sqrt|lambda|, sinc^2(t/2 sqrt|lambda|)
COMPLEX_FUNCS = (0, 1, 7)  # exp(t|lambda|) (G1), exp(t lambda) (G2), sinc(t lambda) (G2 sEWI)


def ref_sinc(x):  # eigen_krylov_real.hpp:95-97 (and matfunc_complex.hpp:293-300 for complex x)
    small = np.abs(x) < 1e-8
    return np.where(small, 1.0, np.sin(x) / np.where(small, 1.0, x))


def ref_f(func, lam, t):
    """f(lambda) of every convention (eigen_krylov_complex.hpp:71-77, eigen_krylov_real.hpp:53-201,
    nlsolvers/host/include/eigen_krylov_complex.hpp:67-72, matfunc_complex.hpp:290-300)."""
    if func == 0:
        return np.exp(t * np.abs(lam))
    if func == 1:
        return np.exp(t * lam)
    if func == 7:
        return ref_sinc(t * lam.astype(complex))
    t = float(np.real(t))
    x = t * np.sqrt(np.abs(lam))
    return {2: lambda: np.cos(x), 3: lambda: ref_sinc(x), 4: lambda: ref_sinc(x) ** 2,
            5: lambda: x, 6: lambda: ref_sinc(t / 2 * np.sqrt(np.abs(lam))) ** 2}[func]()


def ref_eig(d, m):
    """The m x m matrix the eigensolver sees (lower triangle, real diagonal:
    eigen_krylov_complex.hpp:69, eigen_krylov_real.hpp:69) and its eigenpairs."""
    T = d[f"T{m}"]
    H = np.tril(T, -1) + np.tril(T, -1).conj().T + np.diag(T.diagonal().real)
    return np.linalg.eigh(H)


def ref_action(d, m, t, func=0, V=None):
    """beta0 V Q f(Lambda) Q^H e1 from the reference's own V and T
    (eigen_krylov_complex.hpp:69-83, eigen_krylov_real.hpp:69-84)."""
    lam, Q = ref_eig(d, m)
    V = d["V16"][:m] if V is None else V
    y = float(d["beta0"]) * (V.T @ (Q @ (ref_f(func, lam, t) * Q[0].conj())))
    return y.real if np.isrealobj(V) else y


def ref_kappa(d, m, t, func):
    """The argument scale of f: |t| rho(T), or |t| sqrt(rho(T)) for the sqrt functions."""
    rho = np.abs(ref_eig(d, m)[0]).max()
    return abs(t) * (np.sqrt(rho) if func in REAL_FUNCS else rho)


def ref_action_err(got, ref):
    """rel-L2 of an action, scaled by max|ref| first (sinc(t lambda) of an imaginary
    argument grows like sinh: at kappa ~ 480 its entries are finite but the norm overflows)."""
    sc = np.abs(ref).max()
    return rel_l2(got / sc, ref / sc)


def ref_overflows(ref):
    """The reference's own action is not finite (sinc(t lambda) = sinh(|t lambda|)/|t lambda|
    past ~710): there is nothing to compare but the overflow itself."""
    return not np.all(np.isfinite(ref))


def ref_cases(name):
    """(t, func) pairs checked on a fixture: the real t sqrt|lambda| functions at the
    Gautschi steps' dt (sg_driver_dev.cpp: 5/500) and 10x; the complex conventions at
    t = -i dt (dt = 1e-3, the NLSE configs) and 10x; sinc(t lambda) of an imaginary
    argument only where it is finite (sinh growth)."""
    real = "_real" in name
    ts = (1e-2, 1e-1) if real else (-1e-3j, -1e-2j)
    return [(t, f) for t in ts for f in (REAL_FUNCS if real else COMPLEX_FUNCS)]


@pytest.mark.parametrize("name", REF_LANCZOS)
@pytest.mark.parametrize("m", [10, 16])
def test_ref_lanczos_recurrence(name, m):
    """The oracle's lanczos_L (complex eigen_krylov_complex.hpp:10-53, real
    eigen_krylov_real.hpp:5-51) against the reference's LanczosStepTorch, driven with
    buf1 = L V[j] from the triplet builder: every T entry, every beta, every V row."""
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    dim, n, dx = int(d["dim"]), int(d["n"]), float(d["dx"])
    g = O.grid(dim, n, n, n, dx, dx)
    real = "_real" in name
    V, T, b0 = (O.lanczos_r if real else O.lanczos_c)(g, d["u"], m)
    Tr = d[f"T{m}"]
    assert np.isrealobj(Tr) == real
    scale = np.abs(Tr).max()
    assert np.abs(np.tril(T) - np.tril(Tr)).max() <= TOL_REF_T * scale
    assert np.abs(T - Tr).max() <= TOL_REF_T * scale  # the fresh-dot upper entries too
    assert T[m - 1, m - 1] == 0 and Tr[m - 1, m - 1] == 0  # never written
    beta = np.array([T[j + 1, j].real for j in range(m - 1)])
    assert np.all(np.abs(beta - d[f"beta{m}"]) <= TOL_REF_T * np.abs(d[f"beta{m}"]))
    assert abs(b0 - float(d["beta0"])) <= 1e-15 * b0
    Vr = d["V16"][:m]
    assert max(np.linalg.norm(V[k] - Vr[k]) for k in range(m)) <= TOL_REF_V


@pytest.mark.parametrize("name", REF_LANCZOS)
@pytest.mark.parametrize("m", [10, 16])
def test_ref_krylov_action(name, m):
    """Krylov actions built from the reference's V and T == the oracle's (complex: G1
    exp(t|lambda|), G2 exp(t lambda), sinc(t lambda); real: cos, sinc, sinc^2, id and
    sinc^2-half of t sqrt|lambda|), within TOL_REF_ACT_K (1 + kappa)."""
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    dim, n, dx = int(d["dim"]), int(d["n"]), float(d["dx"])
    g = O.grid(dim, n, n, n, dx, dx)
    real = "_real" in name
    checked = overflow = 0
    for t, func in ref_cases(name):
        kap = ref_kappa(d, m, t, func)
        got = O.krylov_r(g, d["u"], t, m, func) if real else O.krylov_c(g, d["u"], t, m, func)
        with np.errstate(all="ignore"):
            ref = ref_action(d, m, t, func)
        if ref_overflows(ref):
            # (sinc of an imaginary t lambda past kappa ~ 710): the oracle overflows too
            assert func == 7 and not np.all(np.isfinite(got)), (t, func, kap)
            overflow += 1
            continue
        err = ref_action_err(got, ref)
        assert err <= TOL_REF_ACT_K * (1 + kap), (t, func, err, kap)
        checked += 1
    assert checked >= len(ref_cases(name)) - 2  # at most the two sinc(t lambda) cases overflow


def test_ref_neumann_bc_2d():
    """The oracle's BC (complex and real) == the reference's neumann_bc, bit for bit, on
    a square and a non-square field (tensor axis 0 = rows of our [ny][nx] layout)."""
    d = np.load(os.path.join(GOLD, "ref_bc2d.npz"))
    for a, b in ((24, 24), (9, 13)):
        g = O.grid(2, b, a, 1, 1.0, 1.0)
        uc, ur = d[f"uc_{a}x{b}"], d[f"ur_{a}x{b}"]
        assert np.array_equal(O.neumann_bc(g, uc.ravel()).reshape(a, b), d[f"bc_c_{a}x{b}"])
        assert np.array_equal(O.neumann_bc_r(g, ur.ravel()).reshape(a, b), d[f"bc_r_{a}x{b}"])
        assert np.array_equal(np_ref.neumann_bc(2, b, a, 1, uc.ravel()).reshape(a, b), d[f"bc_c_{a}x{b}"])
