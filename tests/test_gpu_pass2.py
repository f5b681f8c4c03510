"""GPU parity of the two-vectors-per-pass Lanczos (NLS_PASS2=1, nls_pass2.hpp,
nls_pass2d.hpp): 3D isotropic NLSE trajectories against the CPU oracle, with the
same tolerances as tests/test_gpu_parity.py, for the LDS-DMA pass k_p2d.  Every
run ends each basis in the fused tail (k_alpha_l2 over S_{m-2}, k_p2tail, k_tail).
k_p2d takes 4-row tiles (ny % 4 == 0) and m <= 18; other shapes run the one-vector
passes."""
import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2
from test_gpu_parity import soliton_field, spacing

pytestmark = pytest.mark.gpu

nls_amd = pytest.importorskip("nls_amd")

TOL_KRYLOV, TOL_TRAJ = 1e-12, 1e-10


@pytest.fixture(autouse=True)
def _pass2(monkeypatch):
    """The two-vector passes (k_p2d) with several z chunks per column of tiles."""
    monkeypatch.setenv("NLS_PASS2", "1")
    monkeypatch.setenv("NLS_P2_KZ", "8")


def _eligible(nx, ny, m):
    """Does the handle run the two-vector pass (nls_api.cpp alloc_all)?  k_p2d for
    ny % 4 == 0 and m <= 18, the register form k_lap + k_p2m (nls_pass2g.hpp) for the other
    complex shapes up to m = 30."""
    return 3 <= m <= 30


def _form(nx, ny, m):
    return "dma" if ny % 4 == 0 and m <= 18 else "reg"


def _ran_pass2(s, m):
    """s-step pass launches are timed at their start J (0, 2, 4, ...); the plain path
    times every j."""
    t = s.timing()
    cnt = t["update_count"]
    return cnt[0] > 0 and cnt[1] == 0  # s-step passes start at J = 0, 2, (5,) ... never at 1


@pytest.mark.parametrize("nx,ny,nz,m", [(64, 16, 12, 16), (64, 32, 20, 10), (128, 16, 9, 15),
                                        (64, 16, 16, 25), (64, 16, 10, 3), (64, 48, 8, 4),
                                        (64, 20, 11, 18), (50, 12, 13, 16), (130, 8, 9, 5),
                                        (40, 18, 10, 16), (33, 7, 9, 12), (24, 24, 24, 30)])
@pytest.mark.parametrize("eq", [0, 1])
def test_pass2_trajectory_matches_oracle(nx, ny, nz, m, eq):
    L = 10.0
    dx = spacing(nx, L)
    u0 = soliton_field(3, nx, ny, nz, L, seed=11)
    u0 = u0 / np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** 3)
    g = O.grid(3, nx, ny, nz, dx, dx)
    dt, nsteps = 1e-3, 10
    ref = O.nlse_steps(g, u0, dt, nsteps, m, nonlin=eq)
    with nls_amd.Solver(3, nx, ny, nz, dx, dx, equation=eq, m=m) as s:
        s.set_field(u0)
        s.set_timing(True)
        s.step(dt, nsteps)
        u = s.get_field()
        assert _ran_pass2(s, m) == _eligible(nx, ny, m)
    assert np.all(np.isfinite(u))
    assert rel_l2(u, ref) <= TOL_TRAJ


@pytest.mark.parametrize("L", [10.0, 0.6])  # ||L|| ~ 1e2 and ~ 3e4 (the 512^3 bench's dx is 0.039)
def test_pass2_one_step_matches_plain_path(monkeypatch, L):
    nx, ny, nz, m = 64, 32, 16, 16
    dx = spacing(nx, L)
    u0 = soliton_field(3, nx, ny, nz, L, seed=5)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("NLS_PASS2", mode)
        with nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m) as s:
            s.set_field(u0)
            s.step(1e-3, 1)
            out[mode] = s.get_field()
    assert rel_l2(out["1"], out["0"]) <= 1e-12


@pytest.mark.parametrize("eq", [0, 1])
def test_multi_step_call_equals_single_steps(eq):
    """The NLSE tail writes u only on the last step of an nls_step call (the other steps
    write just the next start vector): one 5-step call equals five 1-step calls bitwise."""
    nx, ny, nz, m = 64, 16, 12, 16
    dx = spacing(nx, 10.0)
    u0 = soliton_field(3, nx, ny, nz, 10.0, seed=3)
    out = []
    for calls in ((5,), (1, 1, 1, 1, 1), (2, 3)):
        with nls_amd.Solver(3, nx, ny, nz, dx, dx, equation=eq, m=m) as s:
            s.set_field(u0)
            for k in calls:
                s.step(1e-3, k)
            out.append(s.get_field())
    assert np.array_equal(out[0], out[1]) and np.array_equal(out[0], out[2])


# ---- 2D: k_p2d on planes of 4 rows (nls_api.cpp p2_geo; one rank, ny % 4 == 0) ----


def _eligible2d(ny, m):
    return 3 <= m <= 30  # k_p2d on planes of 4 rows (ny % 4 == 0, ny >= 8, m <= 18), else k_lap + k_p2m


@pytest.mark.parametrize("nx,ny,m", [(64, 64, 16), (300, 20, 10), (50, 12, 16), (130, 8, 5), (70, 66, 16),
                                     (64, 40, 3), (96, 36, 17)])
@pytest.mark.parametrize("eq", [0, 1])
def test_pass2_2d_trajectory_matches_oracle(nx, ny, m, eq):
    """The 2D row neighbours are the march's row wrap across planes of 4 rows; the plane
    neighbours are dropped; boundary rows are 2D rows 0 and ny-1 (x edges as in 3D)."""
    L = 10.0
    dx = spacing(nx, L)
    dy = spacing(ny, L)
    u0 = soliton_field(2, nx, ny, 1, L, seed=12)
    u0 = u0 / np.sqrt(np.sum(np.abs(u0) ** 2) * dx * dy)
    g = O.grid(2, nx, ny, 1, dx, dy)
    dt, nsteps = 1e-3, 10
    ref = O.nlse_steps(g, u0, dt, nsteps, m, nonlin=eq)
    with nls_amd.Solver(2, nx, ny, 1, dx, dy, equation=eq, m=m) as s:
        s.set_field(u0)
        s.set_timing(True)
        s.step(dt, nsteps)
        u = s.get_field()
        if m > 3:  # at m = 3 both paths launch one update at J = 0: not telling
            assert _ran_pass2(s, m) == _eligible2d(ny, m)
    assert np.all(np.isfinite(u))
    assert rel_l2(u, ref) <= TOL_TRAJ


@pytest.mark.parametrize("n", [256, 512])
def test_pass2_2d_stiff_matches_oracle(n):
    """C2's spacing (dx = 20/4095, ||L|| dt ~ 1.7e2) on a grid the oracle runs in seconds."""
    dx = 20.0 / 4095
    u0 = soliton_field(2, n, n, 1, n * dx / 2, seed=13)
    g = O.grid(2, n, n, 1, dx, dx)
    ref = O.nlse_steps(g, u0, 1e-3, 6, 16)
    with nls_amd.Solver(2, n, n, 1, dx, dx, m=16) as s:
        s.set_field(u0)
        s.set_timing(True)
        s.step(1e-3, 6)
        u = s.get_field()
        assert _ran_pass2(s, 16)
    assert rel_l2(u, ref) <= TOL_TRAJ


# ---- real 2D Gautschi (sine-Gordon G1 and the G2 family): k_p2d on cell pairs ----


def _eligible_pr(nx, ny, m):
    return nx % 2 == 0 and nx >= 4 and ny % 4 == 0 and ny >= 8 and m <= 18


@pytest.mark.parametrize("nx,ny,m", [(64, 64, 10), (50, 12, 10), (130, 16, 16), (66, 40, 5), (7, 8, 10),
                                     (30, 22, 10), (96, 36, 3)])
def test_pass2_sg_trajectory_matches_oracle(nx, ny, m):
    """sg_solver_dev.hpp:168-193: two bases per step (id/cos of u, sinc^2 of g(u)), both
    by two-vector passes on cell pairs (the x neighbours cross the pair; real dots =
    the real parts of the pair dots)."""
    L = 3.0
    dx, dy = spacing(nx, L), spacing(ny, L)
    x = np.linspace(-L, L, nx)
    y = np.linspace(-L, L, ny)
    Y, X = np.meshgrid(y, x, indexing="ij")
    rng = np.random.default_rng(21)
    u0 = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y))) + 1e-3 * rng.standard_normal(X.shape)).ravel()
    dt = 5.0 / 500
    up0 = u0 - dt * 0.1 * np.sin(X).ravel()
    mf = -np.ones(u0.size)
    g = O.grid(2, nx, ny, 1, dx, dy)
    ref_u, ref_up = O.sg_steps(g, u0, up0, mf, dt, 12, m)
    with nls_amd.Solver(2, nx, ny, 1, dx, dy, equation=nls_amd.SG_GAUTSCHI, m=m) as s:
        s.set_sg_state(u0, up0, mf)
        s.set_timing(True)
        s.step(dt, 12)
        u = s.get_field()
        if m > 3:
            assert _ran_pass2(s, m) == _eligible_pr(nx, ny, m)
    assert rel_l2(u, ref_u) <= TOL_TRAJ


@pytest.mark.parametrize("kind", sorted(O.GG_KINDS))
def test_pass2_gautschi_g2_with_bc_matches_oracle(kind):
    """phi4 / sg_single / sg_double / sg_hyperbolic (G2, m(x), BC after every step)."""
    eq = {"phi4": nls_amd.PHI4, "sg": nls_amd.SG_G2, "sg_double": nls_amd.SG_DOUBLE,
          "sg_hyperbolic": nls_amd.SG_HYPERBOLIC}[kind]
    n, L, m, dt, steps = 40, 4.0, 10, 1e-2, 8
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    rng = np.random.default_rng(22)
    u0 = (1.2 * np.exp(-(X ** 2 + Y ** 2) / 2) + 1e-3 * rng.standard_normal(X.shape)).ravel()
    up = u0 - dt * (0.2 * np.sin(X) * np.exp(-(X ** 2 + Y ** 2) / 4)).ravel()
    mf = (1.0 + 0.2 * np.cos(X + Y)).ravel()
    ref, _ = O.gautschi_g2_steps(O.grid(2, n, n, 1, dx, dx), O.GG_KINDS[kind], u0, up, mf, dt, steps, m)
    with nls_amd.Solver(2, n, n, 1, dx, dx, equation=eq, m=m) as s:
        s.set_sg_state(u0, up, mf)
        s.set_timing(True)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        u = s.get_field()
        assert _ran_pass2(s, m)
    assert rel_l2(u, ref) <= TOL_TRAJ


def test_pass2_sg_stiff_matches_oracle():
    """C4's spacing (dx = 6/8191) on 256^2."""
    n, dx, m, dt = 256, 6.0 / 8191, 10, 5.0 / 500
    x = (np.arange(n) - n / 2) * dx
    Y, X = np.meshgrid(x, x, indexing="ij")
    u0 = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y) / (n * dx / 6)))).ravel()
    g = O.grid(2, n, n, 1, dx, dx)
    ref_u, _ = O.sg_steps(g, u0, u0.copy(), -np.ones(u0.size), dt, 4, m)
    with nls_amd.Solver(2, n, n, 1, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=m) as s:
        s.set_sg_state(u0, u0.copy(), -np.ones(u0.size))
        s.set_timing(True)
        s.step(dt, 4)
        u = s.get_field()
        assert _ran_pass2(s, m)
    assert rel_l2(u, ref_u) <= TOL_TRAJ


@pytest.mark.parametrize("dim,nx,ny,nz,m,large", [(3, 64, 16, 12, 16, "0"), (3, 64, 32, 20, 10, "1"),
                                                   (3, 130, 8, 9, 5, "0"), (2, 256, 64, 1, 16, "0"),
                                                   (3, 64, 16, 16, 4, "1")])
def test_fused_colsum_p2coef_bitwise_equal_separate(monkeypatch, dim, nx, ny, nz, m, large):
    """NLS_P2_FUSE=1 (k_colsum_p2coef: the pass's column sums and its coefficient step in
    one launch, the last workgroup running k_p2coef) against the two launches: the same
    per-column summation order, so the trajectory is the same bits."""
    L = 10.0
    dx = spacing(nx, L)
    u0 = soliton_field(dim, nx, ny, nz, L, seed=17)
    monkeypatch.setenv("NLS_LARGE_SLAB", large)
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("NLS_P2_FUSE", fuse)
        with nls_amd.Solver(dim, nx, ny, nz if dim == 3 else 1, dx, dx, m=m) as s:
            s.set_field(u0)
            s.step(1e-3, 3)
            s.step(1e-3, 2)
            out[fuse] = s.get_field()
    assert np.all(np.isfinite(out["1"]))
    assert np.array_equal(out["1"].view(np.uint64), out["0"].view(np.uint64))
