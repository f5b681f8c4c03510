"""GPU parity of the G2 stepper (nlsolvers/device/include/nlse_dev.hpp behind
nlse_cubic_driver_{2d,3d}.cpp) against the CPU oracle, through the C-ABI.

G2 differs from G1 in every part of the step: the
operator is div(c grad) with face-averaged c (laplacians.hpp:54-218), the
nonlinear phase is exp(+tau/2 m(x)|u|^2), the linear flow is exp(tau*lambda)
(no |.|), and the drivers apply the Neumann copy BC after every step.

Tolerances: stencil apply <= 1e-14, one Krylov action <= 1e-12, trajectories
<= 1e-10 (north_star's bound), BC bit-exact (it is a copy).
"""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(os.path.dirname(HERE), "nonlinear-solvers_amd", "bin")
GOLD = os.path.join(HERE, "golden")
TOL_OP, TOL_KRYLOV, TOL_TRAJ = 1e-14, 1e-12, 1e-10


def fields(dim, nx, ny, nz, seed=0, L=4.0):
    """u0 (a few Gaussian bumps + noise), m(x) > 0 focusing, c(x) in [0.5, 1.5]."""
    rng = np.random.default_rng(seed)
    shp = (ny, nx) if dim == 2 else (nz, ny, nx)
    axes = [np.linspace(-L, L, s) for s in shp]
    grids = np.meshgrid(*axes, indexing="ij")
    r2 = sum(g * g for g in grids)
    u = np.exp(-r2) * np.exp(1j * grids[-1]) + 0.4 * np.exp(-sum((g - 1.0) ** 2 for g in grids))
    u = u.ravel() + 1e-3 * (rng.standard_normal(u.size) + 1j * rng.standard_normal(u.size))
    c = 1.0 + 0.5 * np.sin(0.7 * grids[-1] + 0.3 * grids[0]).ravel() * rng.uniform(0.5, 1.0, u.size)
    mf = 1.0 + 0.5 * np.cos(grids[0]).ravel()
    return u, mf, c


GRIDS = [  # (dim, nx, ny, nz)
    (2, 32, 32, 1),
    (2, 300, 20, 1),     # two partial x-tiles
    (2, 7, 5, 1),
    (3, 12, 12, 12),
    (3, 70, 9, 11),      # partial x / y tiles, several z chunks, y-wrap across planes
    (3, 5, 6, 3),
]


def solver(dim, nx, ny, nz, dx, m, **kw):
    return nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_G2, m=m, **kw)


def set_form(monkeypatch, form):
    """Two-vector pass form of the G2 operator: "dma" (k_p2d with the c field staged
    beside S_J, nls_pass2a.hip; where the grid allows it), "reg" (the register form
    k_lap + k_p2m, nls_pass2g.hpp) or "one" (one-vector passes)."""
    monkeypatch.setenv("NLS_PASS2", "0" if form == "one" else "1")
    monkeypatch.setenv("NLS_P2_REG", "1" if form == "reg" else "0")


def dma_form(form, dim, nx, ny, m):
    """Whether the LDS-DMA pass runs (nls_api.cpp alloc_all: 3D, ny % 4 == 0, nx even, m <= 26)."""
    return form == "dma" and dim == 3 and ny % 4 == 0 and nx % 2 == 0 and nx >= 4 and m <= 26


def check_form(cnt, form, dim, nx, ny, m, runs):
    """update_count[0] = J = 0 passes: one launch each in the DMA form, two (y = L S_0,
    then the pass) in the register form; the two-vector passes start at even J only."""
    if form == "one":
        assert cnt[1] > 0
        return
    assert cnt[1] == 0
    assert cnt[0] == (runs if dma_form(form, dim, nx, ny, m) else 2 * runs), cnt[:4]


@pytest.mark.parametrize("dim,nx,ny,nz", GRIDS)
def test_aniso_laplacian_matches_oracle(dim, nx, ny, nz):
    dx = 0.37
    u, mf, c = fields(dim, nx, ny, nz, seed=1)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ref = O.laplacian_aniso_c(g, c, u)
    with solver(dim, nx, ny, nz, dx, 4) as s:
        s.set_coefficients(mf, c)
        y = s.laplacian(u)
    assert rel_l2(y, ref) <= TOL_OP


@pytest.mark.parametrize("dim,nx,ny,nz", GRIDS)
@pytest.mark.parametrize("m", [1, 2, 10, 25])
def test_g2_exp_action_matches_oracle(dim, nx, ny, nz, m):
    """exp(t*lambda) with t = +1j*dt (nlsolvers/device/include/matfunc_complex.hpp:281-287)."""
    dx = 8.0 / (nx - 1)
    u, mf, c = fields(dim, nx, ny, nz, seed=2)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    m = min(m, nx * ny * nz)
    with solver(dim, nx, ny, nz, dx, m) as s:
        s.set_coefficients(mf, c)
        for t in (1e-3j, 1e-2j):
            ref = O.krylov_aniso_c(g, c, u, t, m, nls_amd.F_EXP)
            assert rel_l2(s.krylov_apply(u, t, nls_amd.F_EXP), ref) <= TOL_KRYLOV


@pytest.mark.parametrize("dim,nx,ny,nz", GRIDS)
def test_neumann_bc_bit_exact(dim, nx, ny, nz):
    u, mf, c = fields(dim, nx, ny, nz, seed=3)
    g = O.grid(dim, nx, ny, nz, 0.5, 0.5)
    with solver(dim, nx, ny, nz, 0.5, 4) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        s.apply_bc()
        assert np.array_equal(s.get_field(), O.neumann_bc(g, u))


@pytest.mark.parametrize("form", ["dma", "reg", "one"])
@pytest.mark.parametrize("dim,nx,ny,nz,m", [(2, 32, 32, 1, 20), (2, 300, 20, 1, 20), (3, 12, 12, 12, 25),
                                            (3, 70, 9, 11, 25), (3, 16, 16, 16, 10), (2, 7, 5, 1, 20),
                                            (3, 130, 8, 20, 25), (3, 66, 12, 9, 16)])
def test_g2_trajectory_with_bc_matches_oracle(monkeypatch, form, dim, nx, ny, nz, m):
    """The driver loop (nlse_cubic_driver_3d.cpp:116-119): step, then apply_bc.  With
    the two-vector passes in both forms (set_form: the LDS-DMA pass with c staged
    beside S_J, the default where the grid allows it, and the register form) and with
    the one-vector passes.  130 x 8 x 20: a ragged third x tile, two y tiles, the
    y-wrap across tile and plane edges."""
    set_form(monkeypatch, form)
    L, dt, steps = 4.0, 1e-3, 12
    dx = 2 * L / (nx - 1)
    u, mf, c = fields(dim, nx, ny, nz, seed=4)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    m = min(m, nx * ny * nz)
    ref = O.nlse_g2_steps(g, c, mf, u, dt, steps, m, bc=True)
    ref_nobc = O.nlse_g2_steps(g, c, mf, u, dt, steps, m, bc=False)
    with solver(dim, nx, ny, nz, dx, m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        s.set_timing(True)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
        check_form(s.timing()["update_count"], form, dim, nx, ny, m, steps)
        s.set_timing(False)
        s.set_field(u)
        s.step(dt, steps)
        out_nobc = s.get_field()
    assert rel_l2(out, ref) <= TOL_TRAJ
    assert rel_l2(out_nobc, ref_nobc) <= TOL_TRAJ


@pytest.mark.parametrize("eq,form", [("g2", "dma"), ("g2", "reg"), ("g2_2d", "reg")])
def test_g2_stiff_two_vector_matches_oracle(monkeypatch, eq, form):
    """The G2 production workload's spacing (bench g2_3d_256: L = 10, dx = 20/255, m = 25;
    nlse_cubic_driver_3d.cpp:112-114) on a 48^3 sub-grid, 2D at m = 20 on 256^2 with the
    2D driver's spacing; two-vector passes in both forms (3D), BC after every step, 10 steps."""
    set_form(monkeypatch, form)
    dim = 3 if eq == "g2" else 2
    n, m = (48, 25) if dim == 3 else (256, 20)
    dx, dt, steps = 20.0 / 255, 1e-3, 10
    u, mf, c = fields(dim, n, n, n, seed=9, L=(n - 1) * dx / 2)
    g = O.grid(dim, n, n, n, dx, dx)
    ref = O.nlse_g2_steps(g, c, mf, u, dt, steps, m, bc=True)
    with solver(dim, n, n, n, dx, m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        s.set_timing(True)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
        cnt = s.timing()["update_count"]
        # two-vector passes at even J only, the last at J = m - 4 or m - 3
        check_form(cnt, form, dim, n, n, m, steps)
        assert max(j for j in range(32) if cnt[j]) >= m - 4
    assert rel_l2(out, ref) <= TOL_TRAJ


def test_g2_snapshot_is_pre_bc():
    """step() stores the snapshot before the driver's apply_bc (nlse_dev.hpp:195-197)."""
    dim, n, m, dt = 3, 10, 12, 1e-3
    dx = 0.8
    u, mf, c = fields(dim, n, n, n, seed=5)
    g = O.grid(dim, n, n, n, dx, dx)
    with solver(dim, n, n, n, dx, m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        s.step(dt, 1)
        pre = s.get_field()
        s.apply_bc()
        post = s.get_field()
        s.step(dt, 1)
        nxt = s.get_field()
    ref_pre = O.nlse_g2_steps(g, c, mf, u, dt, 1, m, bc=False)
    assert rel_l2(pre, ref_pre) <= TOL_TRAJ
    assert np.array_equal(post, O.neumann_bc(g, pre))
    assert rel_l2(nxt, O.nlse_g2_steps(g, c, mf, O.neumann_bc(g, ref_pre), dt, 1, m, bc=False)) <= TOL_TRAJ


@pytest.mark.parametrize("name", ["g2_3d", "g2_2d"])
def test_g2_golden_fixture(name):
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    n, dim, m, dt = int(d["n"]), int(d["dim"]), int(d["m"]), float(d["dt"])
    with solver(dim, n, n, n, float(d["dx"]), m) as s:
        s.set_coefficients(d["mfield"], d["c"])
        s.set_field(d["u0"])
        for _ in range(int(d["steps"])):
            s.step(dt, 1)
            s.apply_bc()
        assert rel_l2(s.get_field(), d["u"]) <= TOL_TRAJ


def test_g2_state_errors():
    with solver(3, 8, 8, 8, 0.5, 4) as s:
        s.set_field(np.ones(512, complex))
        with pytest.raises(nls_amd.NlsError) as e:
            s.step(1e-3)
        assert e.value.code == -6 and "set_coefficients" in str(e.value)
    with nls_amd.Solver(3, 8, 8, 8, 0.5, m=4) as s:
        with pytest.raises(nls_amd.NlsError) as e:
            s.set_coefficients(np.ones(512), np.ones(512))
        assert e.value.code == -6


@pytest.mark.parametrize("dim,n,nranks", [(3, 16, 2), (3, 13, 3), (2, 40, 4)])
def test_g2_slabs_match_single_rank(dim, n, nranks):
    """z-slab decomposition (local transport): c halo exchanged once, BC across
    the boundary slabs, W_0 refresh + halo after the BC."""
    m, dt, steps = 12, 1e-3, 6
    dx = 8.0 / (n - 1)
    u, mf, c = fields(dim, n, n, n, seed=6)
    P = n * n if dim == 3 else n
    ref = O.nlse_g2_steps(O.grid(dim, n, n, n, dx, dx), c, mf, u, dt, steps, m, bc=True)
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            s = solver(dim, n, n, n, dx, m, device=0, nranks=nranks, rank=r, group=grp)
            sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
            s.set_coefficients(mf[sl], c[sl])
            s.set_field(u[sl])
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            out[r] = s.get_field()
            s.close()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    assert rel_l2(np.concatenate(out), ref) <= TOL_TRAJ


@pytest.mark.parametrize("form", ["dma", "reg"])
@pytest.mark.parametrize("dim,n,nranks", [(3, 16, 2), (3, 13, 3), (2, 40, 2)])
def test_sewi_slabs_match_single_rank(monkeypatch, form, dim, n, nranks):
    """sEWI (three Krylov actions per step on one basis, run_lanczos2 on collective
    handles: two-plane halos, the basis re-warmed for each action) on 2-3 z-slabs of
    the in-process group == the single-rank GPU run == the oracle.  3D n = 16 takes the
    LDS-DMA pass (ny % 4 == 0), n = 13 and 2D the register form."""
    set_form(monkeypatch, form)
    m, dt, steps = 15, 1e-3, 4
    dx = 8.0 / (n - 1)
    u, mf, c = fields(dim, n, n, n, seed=12)
    P = n * n if dim == 3 else n
    g = O.grid(dim, n, n, n, dx, dx)
    ref, _ = O.nlse_sewi_steps(g, c, mf, u, None, dt, 1, steps, m, bc=True)
    with solver(dim, n, n, n, dx, m) as s1:
        s1.set_coefficients(mf, c)
        s1.set_field(u)
        for i in range(1, steps + 1):
            s1.step_sewi(dt, i)
            s1.apply_bc()
        one = s1.get_field()
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            s = solver(dim, n, n, n, dx, m, device=0, nranks=nranks, rank=r, group=grp)
            sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
            s.set_coefficients(mf[sl], c[sl])
            s.set_field(u[sl])
            for i in range(1, steps + 1):
                s.step_sewi(dt, i)
                s.apply_bc()
            out[r] = s.get_field()
            s.close()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    slabs = np.concatenate(out)
    assert rel_l2(one, ref) <= TOL_TRAJ
    assert rel_l2(slabs, ref) <= TOL_TRAJ
    assert rel_l2(slabs, one) <= TOL_TRAJ


@pytest.mark.parametrize("dim", [3, 2])
def test_g2_driver_matches_oracle(tmp_path, dim):
    """nlse_3d_dev / nlse_2d_dev end to end: no normalisation, snapshot 0 = u0,
    snapshots pre-BC every nt/ns steps, BC after each step, m = 25 / 20."""
    n, L, T, nt, ns = (12, 4.0, 0.02, 10, 5) if dim == 3 else (24, 4.0, 0.02, 10, 5)
    m = 25 if dim == 3 else 20
    dx = 2 * L / (n - 1)
    u, mf, c = fields(dim, n, n, n, seed=7, L=L)
    shp = (n,) * dim
    paths = {k: str(tmp_path / f"{k}.npy") for k in ("u0", "m", "c", "out")}
    np.save(paths["u0"], u.reshape(shp))
    np.save(paths["m"], mf.reshape(shp))
    np.save(paths["c"], c.reshape(shp))
    if dim == 3:
        args = [os.path.join(BIN, "nlse_3d_dev"), str(n), str(n), str(n), str(L), str(L), str(L)]
    else:
        args = [os.path.join(BIN, "nlse_2d_dev"), str(n), str(n), str(L), str(L)]
    args += [paths["u0"], paths["out"], str(T), str(nt), str(ns), paths["m"], paths["c"]]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    traj = np.load(paths["out"])
    assert traj.shape == (ns,) + shp and traj.dtype == np.complex128
    g = O.grid(dim, n, n, n, dx, dx)
    dt, freq = T / nt, nt // ns
    cur = u.copy()
    expect = [u.copy()]
    for i in range(1, nt):
        cur = O.nlse_g2_steps(g, c, mf, cur, dt, 1, m, bc=False)
        if i % freq == 0 and len(expect) < ns:
            expect.append(cur.copy())
        cur = O.neumann_bc(g, cur)
    assert np.array_equal(traj[0].ravel(), u)
    for k in range(1, ns):
        assert rel_l2(traj[k].ravel(), expect[k]) <= TOL_TRAJ, k


# ---- sEWI (NLSESolverDevice::step_sewi, nlse_dev.hpp:205-238) ----------------


@pytest.mark.parametrize("dim,nx,ny,nz", GRIDS[:5])
def test_sinc_action_matches_oracle(dim, nx, ny, nz):
    """G2 "sinc": sinc(t*lambda) with real t = dt (matfunc_complex.hpp:290-300)."""
    dx = 8.0 / (nx - 1)
    u, mf, c = fields(dim, nx, ny, nz, seed=8)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    m = min(15, nx * ny * nz)
    with solver(dim, nx, ny, nz, dx, m) as s:
        s.set_coefficients(mf, c)
        for t in (1e-3, 2e-2):
            ref = O.krylov_aniso_c(g, c, u, t, m, nls_amd.F_SINC)
            assert rel_l2(s.krylov_apply(u, t, nls_amd.F_SINC), ref) <= TOL_KRYLOV


@pytest.mark.parametrize("form", ["dma", "reg", "one"])
@pytest.mark.parametrize("dim,nx,ny,nz,m", [(3, 12, 12, 12, 15), (3, 70, 9, 11, 15), (2, 32, 32, 1, 25),
                                            (2, 300, 20, 1, 25), (3, 130, 8, 20, 15)])
def test_sewi_trajectory_matches_oracle(monkeypatch, form, dim, nx, ny, nz, m):
    """The sEWI driver loop (nlse_cubic_sewi_driver_3d.cpp:116-119): step_sewi(i), apply_bc;
    its three Krylov actions per step by the two-vector passes (both forms) or the
    one-vector passes."""
    set_form(monkeypatch, form)
    L, dt, steps = 4.0, 1e-3, 8
    dx = 2 * L / (nx - 1)
    u, mf, c = fields(dim, nx, ny, nz, seed=9)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ref, _ = O.nlse_sewi_steps(g, c, mf, u, None, dt, 1, steps, m, bc=True)
    with solver(dim, nx, ny, nz, dx, m) as s:
        s.set_coefficients(mf, c)
        s.set_field(u)
        for i in range(1, steps + 1):
            s.step_sewi(dt, i)
            s.apply_bc()
        out = s.get_field()
    assert rel_l2(out, ref) <= TOL_TRAJ


@pytest.mark.parametrize("dim,nx,ny,nz,m", [(3, 12, 12, 12, 15), (3, 130, 8, 20, 15), (3, 12, 8, 6, 3),
                                            (3, 16, 12, 10, 4)])
def test_sewi_concurrent_action_bitwise_equal_serial(monkeypatch, dim, nx, ny, nz, m):
    """The third Krylov action of an sEWI step (exp(2 tau L) u_prev) on a second basis and
    stream, concurrently with the first two (nls_api.cpp sewi_concurrent): the same kernels
    on the same inputs, so the trajectory is bit-for-bit the serial order's."""
    monkeypatch.setenv("NLS_PASS2", "1")
    monkeypatch.setenv("NLS_P2_REG", "0")
    L, dt, steps = 4.0, 1e-3, 5
    dx = 2 * L / (nx - 1)
    u, mf, c = fields(dim, nx, ny, nz, seed=11)
    out = {}
    for conc in ("1", "0"):
        monkeypatch.setenv("NLS_SEWI_CONCURRENT", conc)
        with solver(dim, nx, ny, nz, dx, m) as s:
            s.set_coefficients(mf, c)
            s.set_field(u)
            for i in range(1, steps + 1):
                s.step_sewi(dt, i)
                s.apply_bc()
            out[conc] = s.get_field()
    assert np.array_equal(out["1"].view(np.uint64), out["0"].view(np.uint64))
    if m <= 4:  # the shortest bases (one / two s-step passes per action) against the oracle too
        g = O.grid(dim, nx, ny, nz, dx, dx)
        ref, _ = O.nlse_sewi_steps(g, c, mf, u, None, dt, 1, steps, m, bc=True)
        assert rel_l2(out["1"], ref) <= TOL_TRAJ


def test_sewi_golden_and_errors():
    d = np.load(os.path.join(GOLD, "sewi_3d.npz"))
    n, m, dt = int(d["n"]), int(d["m"]), float(d["dt"])
    with solver(3, n, n, n, float(d["dx"]), m) as s:
        s.set_coefficients(d["mfield"], d["c"])
        s.set_field(d["u0"])
        with pytest.raises(nls_amd.NlsError) as e:
            s.step_sewi(dt, 2)       # no u_prev yet
        assert e.value.code == -6
        for i in range(1, int(d["steps"]) + 1):
            s.step_sewi(dt, i)
            s.apply_bc()
        assert rel_l2(s.get_field(), d["u"]) <= TOL_TRAJ
    with nls_amd.Solver(3, 8, 8, 8, 0.5, m=4) as s:
        s.set_field(np.ones(512, complex))
        with pytest.raises(nls_amd.NlsError) as e:
            s.step_sewi(1e-3, 1)
        assert e.value.code == -6
    # the Klein-Gordon handle has the same operator but a real field: no sEWI
    with nls_amd.Solver(3, 8, 8, 8, 0.5, equation=nls_amd.KG_GAUTSCHI, m=4) as s:
        s.set_coefficients(np.ones(512), np.ones(512))
        s.set_sg_state(np.ones(512), np.ones(512))
        with pytest.raises(nls_amd.NlsError) as e:
            s.step_sewi(1e-3, 1)
        assert e.value.code == -6


@pytest.mark.parametrize("dim", [3, 2])
def test_sewi_driver_matches_oracle(tmp_path, dim):
    n, L, T, nt, ns = (10, 4.0, 0.02, 10, 5) if dim == 3 else (20, 4.0, 0.02, 10, 5)
    m = 15 if dim == 3 else 25
    dx = 2 * L / (n - 1)
    u, mf, c = fields(dim, n, n, n, seed=10, L=L)
    shp = (n,) * dim
    paths = {k: str(tmp_path / f"{k}.npy") for k in ("u0", "m", "c", "out")}
    np.save(paths["u0"], u.reshape(shp))
    np.save(paths["m"], mf.reshape(shp))
    np.save(paths["c"], c.reshape(shp))
    if dim == 3:
        args = [os.path.join(BIN, "nlse_sewi_3d_dev"), str(n), str(n), str(n), str(L), str(L), str(L)]
    else:
        args = [os.path.join(BIN, "nlse_sewi_2d_dev"), str(n), str(n), str(L), str(L)]
    args += [paths["u0"], paths["out"], str(T), str(nt), str(ns), paths["m"], paths["c"]]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    traj = np.load(paths["out"])
    assert traj.shape == (ns,) + shp
    g = O.grid(dim, n, n, n, dx, dx)
    dt, freq = T / nt, nt // ns
    cur, prev = u.copy(), None
    expect = [u.copy()]
    for i in range(1, nt):
        cur, prev = O.nlse_sewi_steps(g, c, mf, cur, prev, dt, i, 1, m, bc=False)
        if i % freq == 0 and len(expect) < ns:
            expect.append(cur.copy())
        cur = O.neumann_bc(g, cur)
    assert np.array_equal(traj[0].ravel(), u)
    for k in range(1, ns):
        assert rel_l2(traj[k].ravel(), expect[k]) <= TOL_TRAJ, k


# ---- G2 cubic-quintic (nlse_cubic_quintic_dev.hpp:16-95) ----------------------

CQ_S = (1.0, -0.5)


def cq_solver(dim, nx, ny, nz, dx, m, s1=CQ_S[0], s2=CQ_S[1], **kw):
    return nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.NLSE_CQ_G2, m=m,
                          sigma1=(s1, 0.0), sigma2=(s2, 0.0), **kw)


@pytest.mark.parametrize("pass2", ["1", "0"])
@pytest.mark.parametrize("dim,nx,ny,nz,m", [(2, 32, 32, 1, 15), (2, 300, 20, 1, 15), (2, 7, 5, 1, 10),
                                            (3, 12, 12, 12, 15), (3, 70, 9, 11, 15), (3, 64, 16, 12, 16)])
def test_cq_g2_trajectory_with_bc_matches_oracle(monkeypatch, pass2, dim, nx, ny, nz, m):
    """The driver loop (nlse_cubic_quintic_driver_dev.cpp:95-98): step, then apply_bc.
    NLS_PASS2 toggles the two-vector basis passes (3D) against the one-vector path."""
    monkeypatch.setenv("NLS_PASS2", pass2)
    L, dt, steps = 4.0, 1e-3, 10
    dx = 2 * L / (nx - 1)
    u, mf, _ = fields(dim, nx, ny, nz, seed=12)
    g = O.grid(dim, nx, ny, nz, dx, dx)
    m = min(m, nx * ny * nz)
    ref = O.nlse_cq_g2_steps(g, mf, u, dt, steps, m, *CQ_S, bc=True)
    ref_nobc = O.nlse_cq_g2_steps(g, mf, u, dt, steps, m, *CQ_S, bc=False)
    with cq_solver(dim, nx, ny, nz, dx, m) as s:
        s.set_coefficients(mf)
        s.set_field(u)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        out = s.get_field()
        s.set_field(u)
        s.step(dt, steps)
        out_nobc = s.get_field()
    assert rel_l2(out, ref) <= TOL_TRAJ
    assert rel_l2(out_nobc, ref_nobc) <= TOL_TRAJ


def test_cq_g2_golden_fixture_and_errors():
    d = np.load(os.path.join(GOLD, "cq_g2_2d.npz"))
    n, m, dt = int(d["n"]), int(d["m"]), float(d["dt"])
    with cq_solver(2, n, n, 1, float(d["dx"]), m, float(d["s1"]), float(d["s2"])) as s:
        s.set_field(d["u0"])
        with pytest.raises(nls_amd.NlsError) as e:
            s.step(dt)                      # m(x) not uploaded yet
        assert e.value.code == -6
        s.set_coefficients(d["mfield"])
        for _ in range(int(d["steps"])):
            s.step(dt, 1)
            s.apply_bc()
        assert rel_l2(s.get_field(), d["u"]) <= TOL_TRAJ


@pytest.mark.parametrize("dim,n,nranks", [(3, 16, 2), (3, 13, 3)])
def test_cq_g2_slabs_match_single_rank(dim, n, nranks):
    m, dt, steps = 15, 1e-3, 6
    dx = 8.0 / (n - 1)
    u, mf, _ = fields(dim, n, n, n, seed=13)
    P = n * n
    ref = O.nlse_cq_g2_steps(O.grid(dim, n, n, n, dx, dx), mf, u, dt, steps, m, *CQ_S, bc=True)
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            s = cq_solver(dim, n, n, n, dx, m, device=0, nranks=nranks, rank=r, group=grp)
            sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
            s.set_coefficients(mf[sl])
            s.set_field(u[sl])
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            out[r] = s.get_field()
            s.close()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    assert rel_l2(np.concatenate(out), ref) <= TOL_TRAJ


@pytest.mark.parametrize("mcase", ["file", "none", "bad_shape"])
def test_cq_g2_driver_matches_oracle(tmp_path, mcase):
    """nlse_cubic_quintic_dev end to end: 11/12 args, m = 15, snapshot 0 = u0, pre-BC
    snapshots every nt/ns steps, BC after each step; a missing m file means m = 1, a
    wrong-shaped one falls back to m = 1 with the reference's message (:65-85)."""
    n, ny, L, T, nt, ns = 24, 20, 4.0, 0.02, 11, 5
    s1, s2 = 0.8, -0.3
    dx = 2 * L / (n - 1)
    dy = 2 * L / (ny - 1)
    u, mf, _ = fields(2, n, ny, 1, seed=14, L=L)
    paths = {k: str(tmp_path / f"{k}.npy") for k in ("u0", "m", "out")}
    np.save(paths["u0"], u.reshape(ny, n))
    args = [os.path.join(BIN, "nlse_cubic_quintic_dev"), str(n), str(ny), str(L), str(L), str(s1), str(s2),
            paths["u0"], paths["out"], str(T), str(nt), str(ns)]
    if mcase == "file":
        np.save(paths["m"], mf.reshape(ny, n))
        args.append(paths["m"])
    elif mcase == "bad_shape":
        np.save(paths["m"], mf.reshape(ny, n)[:, :-1])
        args.append(paths["m"])
        mf = np.ones_like(mf)
    else:
        mf = np.ones_like(mf)
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    if mcase == "bad_shape":
        assert "Coupling array dimensions mismatch" in r.stderr and "Using default m=1.0" in r.stderr
    assert r.stdout == ""
    traj = np.load(paths["out"])
    assert traj.shape == (ns, ny, n) and traj.dtype == np.complex128
    g = O.grid(2, n, ny, 1, dx, dy)
    dt, freq = T / nt, nt // ns
    cur = u.copy()
    expect = [u.copy()]
    for i in range(1, nt):
        cur = O.nlse_cq_g2_steps(g, mf, cur, dt, 1, 15, s1, s2, bc=False)
        if i % freq == 0 and len(expect) < ns:
            expect.append(cur.copy())
        cur = O.neumann_bc(g, cur)
    assert np.array_equal(traj[0].ravel(), u)
    for k in range(1, ns):
        assert rel_l2(traj[k].ravel(), expect[k]) <= TOL_TRAJ, k
