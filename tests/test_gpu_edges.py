"""GPU edge cases of the Krylov stepper that the trajectory tests do not reach.

* Happy breakdown: a constant field is in the null space of the G2 no-flux
  operator div(c grad), so the Lanczos recurrence breaks down after its first
  vector.  The reference divides by the zero beta
  (eigen_krylov_complex.hpp:47, lanczos_complex.hpp:311 skips the write and
  leaves V stale), we drop the dead directions (inv_or_zero, nls_reduce.hpp);
  the answer is then exactly that of a Krylov space of dimension 1, i.e. the
  oracle run with m = 1, which never divides.
* Near breakdown (G1, whose Laplacian has Dirichlet-like boundary rows and no
  constant null vector): an eigenvector start vector leaves a residual of
  rounding size, which the recurrence must normalise without losing accuracy.
* Exhausted space: m = 32 on grids with fewer cells than m; the Krylov
  approximation is then exact, checked against the dense f(L) from eigh.
* m = 32 (the ABI maximum) on partial-tile grids for every equation, against
  the oracle at the same m.
"""
import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


@pytest.fixture(autouse=True, params=["default", "folded", "onevec"])
def _alpha_mode(request, monkeypatch):
    """Every edge case three times: the default sequence (the two-vector passes for
    the 3D isotropic NLSE), the one-vector passes (NLS_PASS2=0), and those with the
    folded alpha forced on (NLS_FUSED_ALPHA=1), whose near-breakdown fallback
    (k_reduce_qa) these cases reach; the variables are read when a handle is created."""
    if request.param == "folded":
        monkeypatch.setenv("NLS_FUSED_ALPHA", "1")
        monkeypatch.setenv("NLS_PASS2", "0")
    elif request.param == "onevec":
        monkeypatch.setenv("NLS_PASS2", "0")
    yield

TOL = 1e-10


def _const(dim, nx, ny, nz, val):
    return np.full(nx * ny * (nz if dim == 3 else 1), val)


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 12, 11, 10), (2, 40, 33, 1)])
@pytest.mark.parametrize("ccase", ["one", "random"])
def test_constant_field_breakdown_g2(dim, nx, ny, nz, ccase):
    """G2 SS2 + BC and sEWI: exp(tau L) and sinc(dt L) of a constant are exact at m = 1."""
    dx, dt, steps = 0.3, 1e-2, 5
    n = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(3)
    c = np.ones(n) if ccase == "one" else rng.uniform(0.5, 1.5, n)
    mf = np.full(n, 1.3)   # uniform m(x): the field stays constant
    u = _const(dim, nx, ny, nz, 0.5 + 0.25j)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ref = O.nlse_g2_steps(g, c, mf, u, dt, steps, 1, bc=True)
    ref_sewi, _ = O.nlse_sewi_steps(g, c, mf, u, None, dt, 1, steps, 1, bc=True)
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_G2, m=16) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
        s.set_field(u)
        for i in range(1, steps + 1):
            s.step_sewi(dt, i)
            s.apply_bc()
        out_sewi = s.get_field()
    for a, r in ((out, ref), (out_sewi, ref_sewi)):
        assert np.all(np.isfinite(a))
        assert rel_l2(a, r) <= TOL


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 12, 11, 10), (2, 40, 33, 1)])
def test_constant_field_breakdown_kg(dim, nx, ny, nz):
    """KG Gautschi (G2): cos / sinc^2 of a constant state are exact at m = 1."""
    dx, dt, steps = 0.3, 1e-2, 5
    n = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(4)
    u0, up0 = np.full(n, 0.7), np.full(n, 0.69)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    c, mf = rng.uniform(0.5, 1.5, n), np.full(n, 1.1)
    ru, _, _ = O.kg_steps(g, c, mf, u0, up0, dt, steps, 1, bc=True)
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.KG_GAUTSCHI, m=10) as s:
        s.set_coefficients(mf, c)
        s.set_sg_state(u0, up0)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
    assert np.all(np.isfinite(out)) and rel_l2(out, ru) <= TOL


def _dense(apply, n, cplx):
    cols = []
    for k in range(n):
        e = np.zeros(n, complex if cplx else float)
        e[k] = 1.0
        cols.append(apply(e))
    A = np.array(cols).T.real
    assert np.allclose(A, A.T, atol=1e-12 * np.abs(A).max())
    return 0.5 * (A + A.T)


def _fmat(A, f):
    lam, Q = np.linalg.eigh(A)
    return (Q * f(lam)) @ Q.T


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 2, 2, 2), (3, 3, 3, 3), (2, 4, 5, 1), (2, 2, 2, 1)])
def test_krylov_exhausted_space_is_exact_g1(dim, nx, ny, nz):
    dx = 0.7
    n = nx * ny * (nz if dim == 3 else 1)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    rng = np.random.default_rng(6)
    u = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    A = _dense(lambda e: O.laplacian_c(g, e), n, True)
    t = -0.05j
    ref = _fmat(A, lambda lam: np.exp(t * np.abs(lam))) @ u
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, m=32) as s:
        y = s.krylov_apply(u, t, nls_amd.F_EXP_ABS)
    assert rel_l2(y, ref) <= TOL
    if dim == 2:   # real Gautschi functions on the SG handle
        ur = rng.standard_normal(n)
        Ar = _dense(lambda e: O.laplacian_r(g, e), n, False)
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=32) as s:
            for func, f in ((nls_amd.F_COS_SQRT, lambda lam: np.cos(0.3 * np.sqrt(np.abs(lam)))),
                            (nls_amd.F_SINC2_HALF, lambda lam: np.sinc(0.15 * np.sqrt(np.abs(lam)) / np.pi) ** 2)):
                y = s.krylov_apply(ur, 0.3, func)
                assert rel_l2(y, _fmat(Ar, f) @ ur) <= TOL


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 3, 3, 3), (2, 4, 5, 1)])
def test_krylov_exhausted_space_is_exact_g2(dim, nx, ny, nz):
    dx = 0.7
    n = nx * ny * (nz if dim == 3 else 1)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    rng = np.random.default_rng(7)
    c, mf = rng.uniform(0.5, 1.5, n), np.ones(n)
    u = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    A = _dense(lambda e: O.laplacian_aniso_c(g, c, e), n, True)
    t = 0.05j
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_G2, m=32) as s:
        s.set_coefficients(mf, c)
        y = s.krylov_apply(u, t, nls_amd.F_EXP)
        ys = s.krylov_apply(u, 0.05, nls_amd.F_SINC)
    assert rel_l2(y, _fmat(A, lambda lam: np.exp(t * lam)) @ u) <= TOL
    assert rel_l2(ys, _fmat(A, lambda lam: np.sinc(0.05 * lam / np.pi)) @ u) <= TOL


M32_GRIDS = [(3, 70, 9, 11), (2, 300, 20, 1)]


@pytest.mark.parametrize("dim,nx,ny,nz", M32_GRIDS)
def test_m32_every_equation(dim, nx, ny, nz):
    """The largest update templates (J = 30) for the iso and aniso tables, complex and real."""
    L, dt, steps, m = 4.0, 1e-3, 3, 32
    dx = 2 * L / (nx - 1)
    n = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(8)
    u = np.exp(-np.linspace(-2, 2, n) ** 2) * (1 + 0.1j) + 1e-2 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    c, mf = rng.uniform(0.5, 1.5, n), rng.uniform(0.5, 1.5, n)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ref = O.nlse_steps(g, u, dt, steps, m)
    ref_cq = O.nlse_steps(g, u, dt, steps, m, nonlin=1)
    ref_g2 = O.nlse_g2_steps(g, c, mf, u, dt, steps, m, bc=True)
    ref_sewi, _ = O.nlse_sewi_steps(g, c, mf, u, None, dt, 1, steps, m, bc=True)
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, m=m) as s:
        s.set_field(u)
        s.step(dt, steps)
        assert rel_l2(s.get_field(), ref) <= TOL
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_CQ, m=m) as s:
        s.set_field(u)
        s.step(dt, steps)
        assert rel_l2(s.get_field(), ref_cq) <= TOL
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_G2, m=m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        assert rel_l2(s.get_field(), ref_g2) <= TOL
        s.set_field(u)
        for i in range(1, steps + 1):
            s.step_sewi(dt, i)
            s.apply_bc()
        assert rel_l2(s.get_field(), ref_sewi) <= TOL
    ur = u.real.copy()
    up = ur - dt * 0.1 * np.sin(np.arange(n))
    ru, _, _ = O.kg_steps(g, c, mf, ur, up, dt, steps, m, bc=True)
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.KG_GAUTSCHI, m=m) as s:
        s.set_coefficients(mf, c)
        s.set_sg_state(ur, up)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        assert rel_l2(s.get_field(), ru) <= TOL
    if dim == 2:
        rs, _ = O.sg_steps(g, ur, up, -mf, dt, steps, m)
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=m) as s:
            s.set_sg_state(ur, up, -mf)
            s.step(dt, steps)
            assert rel_l2(s.get_field(), rs) <= TOL


def test_minimum_g2_grid():
    """3 cells per dimension: the Neumann copy BC overwrites everything but the centre."""
    dim, n, m, dt, steps = 3, 3, 8, 1e-2, 4
    dx = 0.5
    rng = np.random.default_rng(9)
    u = rng.standard_normal(27) + 1j * rng.standard_normal(27)
    c, mf = rng.uniform(0.5, 1.5, 27), rng.uniform(0.5, 1.5, 27)
    g = O.grid(dim, n, n, n, dx, dx)
    ref = O.nlse_g2_steps(g, c, mf, u, dt, steps, m, bc=True)
    with nls_amd.Solver(dim, n, n, n, dx, dx, equation=nls_amd.NLSE_G2, m=m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
    assert rel_l2(out, ref) <= TOL
    assert np.all(out == out[13])


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 12, 11, 10), (2, 40, 33, 1)])
def test_eigenvector_near_breakdown_g1(dim, nx, ny, nz):
    dx = 0.3
    n = nx * ny * (nz if dim == 3 else 1)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    A = _dense(lambda e: O.laplacian_r(g, e), n, False)
    lam, Q = np.linalg.eigh(A)
    for k in (0, n // 3, n - 1):
        v = Q[:, k]
        u = (0.3 + 0.4j) * v
        t = -0.01j
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, m=16) as s:
            y = s.krylov_apply(u, t, nls_amd.F_EXP_ABS)
        assert np.all(np.isfinite(y))
        assert rel_l2(y, np.exp(t * abs(lam[k])) * u) <= TOL
        if dim == 2:
            with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=10) as s:
                y = s.krylov_apply(v, 0.05, nls_amd.F_COS_SQRT)
            assert rel_l2(y, np.cos(0.05 * np.sqrt(abs(lam[k]))) * v) <= TOL
