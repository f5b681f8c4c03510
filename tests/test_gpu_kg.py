"""GPU parity of the G2 Klein-Gordon Gautschi stepper (nlsolvers/device/include/
kg_single.cuh:49-86 behind kg_driver_dev_{2d,3d}.cpp) against the CPU oracle.

u_tt = div(c grad u) - m u^3: per step a sinc^2(t sqrt|L|) action on g = -m u^3,
a cos(t sqrt|L|) action on u, the Gautschi update, v = (u_new - u)/dt, then the
driver's Neumann copy BC on u.  Tolerances: trajectories (u, u_past) <= 1e-10;
the velocity is a difference quotient (extra factor 1/dt): <= 1e-8.
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
TOL_TRAJ, TOL_V = 1e-10, 1e-8


def kg_fields(dim, nx, ny, nz, L=3.0, seed=0):
    rng = np.random.default_rng(seed)
    shp = (ny, nx) if dim == 2 else (nz, ny, nx)
    g = np.meshgrid(*[np.linspace(-L, L, s) for s in shp], indexing="ij")
    r2 = sum(a * a for a in g)
    u0 = (np.exp(-r2) + 1e-3 * rng.standard_normal(r2.shape)).ravel()
    v0 = (0.1 * np.sin(g[-1]) * np.exp(-r2 / 2)).ravel()
    c = (1.0 + 0.3 * np.sin(0.5 * g[-1] + 0.2 * g[0])).ravel()
    mf = (1.0 + 0.2 * np.cos(g[0])).ravel()
    return u0, v0, mf, c


def kg_solver(dim, nx, ny, nz, dx, m=10, **kw):
    return nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=nls_amd.KG_GAUTSCHI, m=m, **kw)


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 12, 12, 12), (3, 70, 9, 11), (2, 32, 32, 1), (2, 300, 20, 1)])
def test_kg_trajectory_matches_oracle(dim, nx, ny, nz):
    L, dt, steps = 3.0, 5e-3, 10
    dx = 2 * L / (nx - 1)
    u0, v0, mf, c = kg_fields(dim, nx, ny, nz, L, seed=1)
    up0 = u0 - dt * v0
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ru, rup, rv = O.kg_steps(g, c, mf, u0, up0, dt, steps, 10, bc=True)
    with kg_solver(dim, nx, ny, nz, dx) as s:
        s.set_coefficients(mf, c)
        s.set_sg_state(u0, up0)
        for _ in range(steps):
            s.step(dt, 1)
            s.apply_bc()
        u = s.get_field()
        v = s.get_sg_velocity(dt)
    assert rel_l2(u, ru) <= TOL_TRAJ
    assert rel_l2(v, rv) <= TOL_V


def test_kg_golden_fixture_and_velocity_before_bc():
    d = np.load(os.path.join(GOLD, "kg_3d.npz"))
    n, dt = int(d["n"]), float(d["dt"])
    with kg_solver(3, n, n, n, float(d["dx"]), m=int(d["m"])) as s:
        s.set_coefficients(d["mfield"], d["c"])
        s.set_sg_state(d["u0"], d["u0"] - dt * d["v0"])
        for _ in range(int(d["steps"])):
            s.step(dt, 1)
            s.apply_bc()
        assert rel_l2(s.get_field(), d["u"]) <= TOL_TRAJ
        # v is the step's (pre-BC) difference quotient, not (u_bc - u_past)/dt
        assert rel_l2(s.get_sg_velocity(dt), d["v"]) <= TOL_V


def test_kg_errors():
    with kg_solver(3, 8, 8, 8, 0.5) as s:
        s.set_sg_state(np.zeros(512), np.zeros(512))
        with pytest.raises(nls_amd.NlsError) as e:
            s.step(1e-3)
        assert e.value.code == -6          # no coefficients
        s.set_coefficients(np.ones(512), np.ones(512))
        with pytest.raises(nls_amd.NlsError) as e:
            s.step(0.0)
        assert e.value.code == -1


@pytest.mark.parametrize("dim,n,nranks", [(3, 14, 2), (2, 30, 3)])
def test_kg_slabs_match_single_rank(dim, n, nranks):
    L, dt, steps = 3.0, 5e-3, 6
    dx = 2 * L / (n - 1)
    u0, v0, mf, c = kg_fields(dim, n, n, n, L, seed=2)
    up0 = u0 - dt * v0
    P = n * n if dim == 3 else n
    ref = O.kg_steps(O.grid(dim, n, n, n, dx, dx), c, mf, u0, up0, dt, steps, 10, bc=True)[0]
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            s = kg_solver(dim, n, n, n, dx, device=0, nranks=nranks, rank=r, group=grp)
            sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
            s.set_coefficients(mf[sl], c[sl])
            s.set_sg_state(u0[sl], up0[sl])
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


@pytest.mark.parametrize("dim", [3, 2])
def test_kg_driver_matches_oracle(tmp_path, dim):
    n, L, T, nt, ns = (10, 3.0, 0.05, 10, 5) if dim == 3 else (20, 3.0, 0.05, 10, 5)
    dx = 2 * L / (n - 1)
    dt, freq = T / nt, nt // ns
    u0, v0, mf, c = kg_fields(dim, n, n, n, L, seed=3)
    shp = (n,) * dim
    p = {k: str(tmp_path / f"{k}.npy") for k in ("u0", "v0", "m", "c", "tu", "tv")}
    for k, a in (("u0", u0), ("v0", v0), ("m", mf), ("c", c)):
        np.save(p[k], a.reshape(shp))
    if dim == 3:
        args = [os.path.join(BIN, "kg_gautschi_3d_dev"), str(n), str(n), str(n), str(L), str(L), str(L)]
    else:
        args = [os.path.join(BIN, "kg_gautschi_2d_dev"), str(n), str(n), str(L), str(L)]
    tail = [str(T), str(nt), str(ns), p["m"], p["c"]]
    r = subprocess.run(args + [p["u0"], p["v0"], p["tu"], p["tv"]] + tail + (["--true-shape"] if dim == 3 else []),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    tu, tv = np.load(p["tu"]), np.load(p["tv"])
    if dim == 3:
        # default: the reference's header [ns, ny, nx] over the full ns*nz*ny*nx payload
        # (kg_driver_dev_3d.cpp:161-163), byte-identical data to the --true-shape file
        ref_u = str(tmp_path / "ref_u.npy")
        r = subprocess.run(args + [p["u0"], p["v0"], ref_u, str(tmp_path / "ref_v.npy")] + tail,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        with open(ref_u, "rb") as f:
            ver = np.lib.format.read_magic(f)
            hdr_shape, _, dtype = np.lib.format._read_array_header(f, ver)
            payload = np.fromfile(f, dtype=dtype)
        assert hdr_shape == (ns, n, n)
        assert np.array_equal(payload, tu.ravel())
    assert tu.shape == (ns,) + shp and tv.shape == (ns,) + shp
    g = O.grid(dim, n, n, n, dx, dx)
    u, up = u0.copy(), u0 - dt * v0
    eu, ev = [u0], [v0]
    for i in range(1, nt):
        u, up, v = O.kg_steps(g, c, mf, u, up, dt, 1, 10, bc=True)
        if i % freq == 0 and i // freq < ns:
            eu.append(u.copy())
            ev.append(v.copy())
    assert np.array_equal(tu[0].ravel(), u0) and np.array_equal(tv[0].ravel(), v0)
    for k in range(1, ns):
        assert rel_l2(tu[k].ravel(), eu[k]) <= TOL_TRAJ, k
        assert rel_l2(tv[k].ravel(), ev[k]) <= TOL_V, k


def _ran_pass2(s):
    """The s-step passes time their launches at J = 0, 2, ...; the one-vector path at every j."""
    cnt = s.timing()["update_count"]
    return cnt[0] > 0 and cnt[1] == 0


@pytest.mark.parametrize("nx,ny,nz,m,kz", [(12, 12, 12, 10, None), (140, 8, 9, 10, None), (22, 20, 16, 10, "4"),
                                           (64, 16, 10, 16, None), (18, 4, 7, 6, "2"), (30, 12, 8, 3, None)])
def test_kg_pair_passes_match_oracle(monkeypatch, nx, ny, nz, m, kz):
    """3D KG on the s-step passes k_p2d<.., PR, A> (real cells as pairs, div(c grad)):
    ragged x tiles (140 = 70 pairs), one and several z chunks, m = 3 .. 16; against the
    oracle and against the one-vector path (NLS_PASS2=0) of the same handle shape."""
    if kz:
        monkeypatch.setenv("NLS_P2_KZ", kz)
    L, dt, steps = 3.0, 5e-3, 8
    dx = 2 * L / (nx - 1)
    u0, v0, mf, c = kg_fields(3, nx, ny, nz, L, seed=4)
    up0 = u0 - dt * v0
    ru, _, rv = O.kg_steps(O.grid(3, nx, ny, nz, dx, dx), c, mf, u0, up0, dt, steps, m, bc=True)
    res = {}
    for p2 in ("1", "0"):
        monkeypatch.setenv("NLS_PASS2", p2)
        with kg_solver(3, nx, ny, nz, dx, m=m) as s:
            s.set_coefficients(mf, c)
            s.set_sg_state(u0, up0)
            s.set_timing(True)
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            assert _ran_pass2(s) == (p2 == "1")
            res[p2] = (s.get_field(), s.get_sg_velocity(dt))
    for u, v in res.values():
        assert rel_l2(u, ru) <= TOL_TRAJ
        assert rel_l2(v, rv) <= TOL_V
    assert rel_l2(res["1"][0], res["0"][0]) <= TOL_TRAJ


@pytest.mark.parametrize("nx,ny,nz,m", [(12, 12, 12, 10), (140, 8, 9, 10), (64, 16, 10, 16)])
def test_kg_two_streams_bitwise_equal_serial(monkeypatch, nx, ny, nz, m):
    """The two Krylov actions of the s-step KG step on two streams (nls_api.cpp: the sinc^2
    basis on stream2 with its own partial buffers) against the serial order
    (NLS_KG_CONCURRENT=0): the same kernels on the same inputs, bit for bit."""
    L, dt, steps = 3.0, 5e-3, 6
    dx = 2 * L / (nx - 1)
    u0, v0, mf, c = kg_fields(3, nx, ny, nz, L, seed=6)
    up0 = u0 - dt * v0
    res = {}
    for conc in ("1", "0"):
        monkeypatch.setenv("NLS_KG_CONCURRENT", conc)
        with kg_solver(3, nx, ny, nz, dx, m=m) as s:
            s.set_coefficients(mf, c)
            s.set_sg_state(u0, up0)
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            res[conc] = (s.get_field(), s.get_sg_velocity(dt))
    for a, b in zip(res["1"], res["0"]):
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


@pytest.mark.parametrize("n,nranks", [(16, 2), (16, 3)])
def test_kg_pair_passes_slabs_match_single_rank(n, nranks):
    """The cell-pair passes on z-slabs (two ghost planes; in-process local transport)."""
    L, dt, steps = 3.0, 5e-3, 5
    dx = 2 * L / (n - 1)
    u0, v0, mf, c = kg_fields(3, n, n, n, L, seed=5)
    up0 = u0 - dt * v0
    P = n * n
    ref = O.kg_steps(O.grid(3, n, n, n, dx, dx), c, mf, u0, up0, dt, steps, 10, bc=True)[0]
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    ran = [None] * nranks
    err = []

    def work(r):
        try:
            s = kg_solver(3, n, n, n, dx, device=0, nranks=nranks, rank=r, group=grp)
            sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
            s.set_coefficients(mf[sl], c[sl])
            s.set_sg_state(u0[sl], up0[sl])
            s.set_timing(True)
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            out[r] = s.get_field()
            ran[r] = _ran_pass2(s)
            s.close()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    assert all(ran)
    assert rel_l2(np.concatenate(out), ref) <= TOL_TRAJ


def test_kg_timing_on_is_bitwise_and_serial():
    """With per-kernel timing on, the KG step runs its two Krylov actions in the serial order
    (no kernel's events then span the other stream's work) -- bit-identical to
    the untimed two-stream step, and every timed class is a real launch count."""
    nx = ny = nz = 24
    L, dt, steps = 3.0, 5e-3, 4
    dx = 2 * L / (nx - 1)
    u0, v0, mf, c = kg_fields(3, nx, ny, nz, L, seed=8)
    up0 = u0 - dt * v0
    res = {}
    for timed in (False, True):
        with kg_solver(3, nx, ny, nz, dx, m=10) as s:
            s.set_coefficients(mf, c)
            s.set_sg_state(u0, up0)
            s.set_timing(timed)
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            res[timed] = s.get_field()
            if timed:
                t = s.timing()
                assert t["steps"] == steps and t["class_count"]["final"] == 2 * steps
                assert all(v >= 0 for v in t["class_ms"].values())
    assert np.array_equal(res[False].view(np.uint64), res[True].view(np.uint64))


@pytest.mark.parametrize("nx,ny,nz,m", [(12, 12, 12, 10), (64, 16, 10, 16)])
def test_kg_fused_colsum_p2coef_bitwise_equal(monkeypatch, nx, ny, nz, m):
    """The KG step's cell-pair passes with the column sums and k_p2coef in one launch
    (NLS_P2_FUSE=1; one last-workgroup counter per basis, the two bases on two streams)
    against the two launches per pass: bit for bit."""
    L, dt, steps = 3.0, 5e-3, 4
    dx = 2 * L / (nx - 1)
    u0, v0, mf, c = kg_fields(3, nx, ny, nz, L, seed=8)
    up0 = u0 - dt * v0
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("NLS_P2_FUSE", fuse)
        with kg_solver(3, nx, ny, nz, dx, m=m) as s:
            s.set_coefficients(mf, c)
            s.set_sg_state(u0, up0)
            for _ in range(steps):
                s.step(dt, 1)
                s.apply_bc()
            res[fuse] = s.get_field()
    assert np.array_equal(res["1"].view(np.uint64), res["0"].view(np.uint64))
